# The driver's likely invocation (round 3: --steps 20 --warmup 5), ROUNDS times,
# plus the default 200-step line once.   tools/gpu_driver_like.sh TAG ROUNDS
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for r in $(seq $2); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20_$r.log 2>&1 || { echo "bench 20 failed"; tail -20 $O/b20_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('steps 20 warmup 5 r%s us/step %.2f train %.2f' % (sys.argv[2], d['ms_per_step']*1e3, d['train_mode']['ms_per_step']*1e3))" $O/b20_$r.log $r
done
timeout -k 10 300 python bench.py > $O/b200.log 2>&1 || { echo "bench 200 failed"; tail -20 $O/b200.log; exit 1; }
python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('steps 200 warmup 20 us/step %.2f train %.2f' % (d['ms_per_step']*1e3, d['train_mode']['ms_per_step']*1e3))" $O/b200.log
