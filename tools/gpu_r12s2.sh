# r12s2: the driver invocation on the final tree (profiles/r12t_*), three runs
set -o pipefail
O=gpurun_out/r12s2; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/d_$r.log 2>&1 || { echo fail; tail -5 $O/d_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('driver r', sys.argv[2], 'us/step %.2f value %.3e train us/step %.2f' % (d['ms_per_step']*1e3, d['value'], d['train_mode']['ms_per_step']*1e3))" $O/d_$r.log $r
done
