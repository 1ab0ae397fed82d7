set -o pipefail
O=gpurun_out/d9; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/diag_scene.py > $O/scene.log 2>&1 || { tail -30 $O/scene.log; exit 1; }
grep -v amdgpu.ids $O/scene.log | grep -A1 "== WG"
