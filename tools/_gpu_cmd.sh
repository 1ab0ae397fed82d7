set -o pipefail
O=gpurun_out/${1:-d40}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/dbg_grad.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in eth_hotel_synth dense_crowd; do
timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 100 > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 1; }
grep '^{' $O/bench_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"], d["ms_per_step"]*1e3, d["train_mode"]["ms_per_step"]*1e3)'
done
