# r12i: the driver's invocation (20 steps, warm-up 5) with the HIP graph (default) vs direct launches (--no-graph), four interleaved rounds
set -o pipefail
O=gpurun_out/r12i; mkdir -p $O
for r in 1 2 3 4; do for g in graph nograph; do
  x=""; [ $g = nograph ] && x="--no-graph"
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train $x > $O/d_${g}_$r.log 2>&1 || { echo fail; tail -5 $O/d_${g}_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('driver', sys.argv[2], 'us/step %.2f' % (d['ms_per_step']*1e3))" $O/d_${g}_$r.log "$g r$r"
done; done
for g in graph nograph; do x=""; [ $g = nograph ] && x="--no-graph"
  timeout -k 10 120 python bench.py --steps 200 --no-cpu-baseline --no-train $x > $O/s_${g}.log 2>&1 || exit 1
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('200 steps', sys.argv[2], 'us/step %.2f' % (d['ms_per_step']*1e3))" $O/s_${g}.log "$g"
done
