set -o pipefail
O=gpurun_out/${1:-d25}; mkdir -p $O
export TMPDIR=/tmp
G2K_DIAG_FLAGS=-DG2K_DIAG_FEW_STAMPS,-DG2K_DIAG_RECUR_REPEAT,-DG2K_DIAG_SKIP_TILES timeout -k 10 200 python tools/diag_scene.py > $O/scene.log 2>&1 || { tail -30 $O/scene.log; exit 1; }
grep -v amdgpu.ids $O/scene.log | grep -A12 "== WG 255"
