# GPU A/B session: tests of the touched paths, interleaved timing of the
# reference sources (tools/ab_ref: the "orig" variant) against this tree,
# the exit-stamp timelines of both.   tools/gpu_ab.sh TAG [notest] CONFIG...
# (AB_VARIANTS / AB_TL override the timed variants / the timelines)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
if [ "$1" = notest ]; then shift; else
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
fi
for c in "$@"; do
  timeout -k 10 300 python tools/ab_time.py --rounds ${AB_ROUNDS:-5} $c ${AB_VARIANTS:-orig base} > $O/ab_$c.log 2>&1 || { echo "ab $c failed"; tail -20 $O/ab_$c.log; exit 1; }
  grep median $O/ab_$c.log
done
for v in ${AB_TL:-tl_end_orig tl_end}; do
timeout -k 10 200 python tools/ab_time.py eth_hotel_synth $v > $O/$v.log 2>&1 || { echo "$v failed"; tail -20 $O/$v.log; exit 1; }
echo "== $v"; grep -v amdgpu.ids $O/$v.log
done
