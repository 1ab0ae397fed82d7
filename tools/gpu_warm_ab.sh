# The timed graph warmed through its own executable (default) vs a separate
# warm-up graph (G2K_BENCH_WARM=graph), at the driver's --steps 20 --warmup 5,
# interleaved, forward and train.   tools/gpu_warm_ab.sh TAG ROUNDS
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bench_graph_gpu.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in $(seq $2); do for w in exec graph; do
  G2K_BENCH_WARM=$w timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${w}_$r.log 2>&1 || { echo "bench $w failed"; tail -20 $O/${w}_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('warm %s r%s us/step %.2f train %.2f' % (sys.argv[2], sys.argv[3], d['ms_per_step']*1e3, d['train_mode']['ms_per_step']*1e3))" $O/${w}_$r.log $w $r
done; done
