# streams 16 / 20 / 32 at the driver's invocation (20 steps, warm-up 5), three interleaved rounds
set -o pipefail
O=gpurun_out/r11t; mkdir -p $O
for r in 1 2 3; do for s in 16 20 32; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train --streams $s > $O/s${s}_$r.log 2>&1 || { echo fail; tail -5 $O/s${s}_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('streams', sys.argv[2], 'r', sys.argv[3], 'us/step %.2f' % (d['ms_per_step']*1e3))" $O/s${s}_$r.log $s $r
done; done
