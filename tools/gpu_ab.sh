# GPU A/B session: tests of the touched paths, interleaved timing of the
# previous commit's library (tools/ab/libg2k_prev.so) against this tree, one
# stamped timeline.   tools/gpu_ab.sh TAG CONFIG...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for c in "$@"; do
  timeout -k 10 300 python tools/ab_time.py --rounds 5 $c prev base > $O/ab_$c.log 2>&1 || { echo "ab $c failed"; tail -20 $O/ab_$c.log; exit 1; }
  grep median $O/ab_$c.log
done
timeout -k 10 200 python tools/ab_time.py eth_hotel_synth tl_gap > $O/gap.log 2>&1 || { echo "tl_gap failed"; tail -20 $O/gap.log; exit 1; }
grep -E "^median|P0 lead|head 0|frame 17|tl_gap" $O/gap.log
