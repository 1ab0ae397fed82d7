set -o pipefail
O=gpurun_out/${1:-d26}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-420
G2K_NO_DMA16=1 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_nodma16.log 2>&1 || { tail -20 $O/bench_nodma16.log; exit 1; }
grep '^{' $O/bench_nodma16.log | cut -c1-200
G2K_DIAG_FLAGS=-DG2K_DIAG_FEW_STAMPS timeout -k 10 200 python tools/diag_scene.py > $O/scene.log 2>&1 || { tail -30 $O/scene.log; exit 1; }
grep -v amdgpu.ids $O/scene.log | grep -A15 "== WG 255"
