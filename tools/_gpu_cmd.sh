set -o pipefail
O=gpurun_out/${1:-d35}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/dbg_grad.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --steps 100 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python tools/pmc_summary.py $O/trace | head -6
grep '^{' $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"]*1e3, d["train_mode"]["ms_per_step"]*1e3)'
