# Graph replay vs host launches of the timed steps, at the driver's 20 steps
# and at 200: tools/gpu_launch_ab.sh TAG ROUNDS
set -o pipefail
O=gpurun_out/$1; R=$2; mkdir -p $O
for r in $(seq $R); do
for k in 20 200; do
for g in "" "--no-graph"; do
  f=$O/b_${k}${g}_$r.txt
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-train --steps $k --warmup 5 $g > $f 2>&1 || { echo "bench $k $g failed"; tail -20 $f; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[2], 'us/step %.2f' % (d['ms_per_step']*1e3))" $f "steps=$k ${g:-graph} r$r"
done; done; done
