set -o pipefail
O=gpurun_out/${1:-d19}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("BENCH", d["value"], d["ms_per_step"], d["roofline"]["kernel_us"], d["roofline"]["frac"])'
G2K_DIAG_FLAGS=-DG2K_DIAG_FEW_STAMPS timeout -k 10 200 python tools/diag_scene.py > $O/scene.log 2>&1 || { tail -30 $O/scene.log; exit 1; }
grep -v amdgpu.ids $O/scene.log | grep -A5 "== WG 255"
