# GPU_MAX_HW_QUEUES (HIP's hardware queues per process; default 4) with the 16-stream bench
set -o pipefail
O=gpurun_out/r11q; mkdir -p $O
for r in 1 2; do for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train > $O/q${q}_20_$r.log 2>&1 || { echo fail; tail -5 $O/q${q}_20_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('hwq', sys.argv[2], '20 steps us/step %.2f' % (d['ms_per_step']*1e3))" $O/q${q}_20_$r.log $q
done; done
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --steps 200 --no-cpu-baseline --no-train > $O/q${q}_200.log 2>&1 || { echo fail; tail -5 $O/q${q}_200.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('hwq', sys.argv[2], '200 steps us/step %.2f' % (d['ms_per_step']*1e3))" $O/q${q}_200.log $q
done
