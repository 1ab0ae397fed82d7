# Round-4 GPU session: the whole GPU suite (no -x: every failure at once),
# smoke, the default bench line, then the experiments named on the command line.
#   tools/gpu_r4.sh TAG [sweep]   (sweep: the specs in $SWEEP, tools/gpu_sweep.sh)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep FAILED $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc $rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
for x in "$@"; do
case $x in
sweep) bash tools/gpu_sweep.sh ${TAG}_sw 1 $SWEEP || exit 1 ;;
esac
done
