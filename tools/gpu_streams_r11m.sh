# streams sweep at the driver's invocation (20 steps, warm-up 5) and at 200 steps, eth_hotel_synth
set -o pipefail
O=gpurun_out/r11m; mkdir -p $O
for r in 1 2; do for s in 4 6 8 12 16; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train --streams $s > $O/s${s}_20_$r.log 2>&1 || { echo fail; tail -5 $O/s${s}_20_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('20 steps streams', sys.argv[2], 'r', sys.argv[3], 'us/step %.2f' % (d['ms_per_step']*1e3))" $O/s${s}_20_$r.log $s $r
done; done
for s in 4 8 12 16; do
  timeout -k 10 120 python bench.py --steps 200 --no-cpu-baseline --no-train --streams $s > $O/s${s}_200.log 2>&1 || { echo fail; tail -5 $O/s${s}_200.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('200 steps streams', sys.argv[2], 'us/step %.2f' % (d['ms_per_step']*1e3))" $O/s${s}_200.log $s
done
