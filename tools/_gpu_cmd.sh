set -o pipefail
O=gpurun_out/d6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python tools/diag_scene.py > $O/scene.log 2>&1 || { tail -30 $O/scene.log; exit 1; }
grep "== WG" $O/scene.log
timeout -k 10 400 python tools/ab_variants.py --rounds 7 base= > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep median $O/ab.log
