# Round-4 GPU session: the whole GPU suite (no -x: every failure at once),
# smoke, the default bench line, then the experiments named on the command line.
#   tools/gpu_r4.sh TAG [np] [overhead]
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
np) G2K_SCENE_NP=4 timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py tests/test_split_gpu.py -q -m gpu --timeout 120 --timeout-method thread > $O/np4_tests.log 2>&1 || { echo "np4 tests failed"; tail -30 $O/np4_tests.log; exit 1; }
    tail -1 $O/np4_tests.log
    bash tools/gpu_np_ab.sh ${TAG}_np 1 eth_hotel_synth eth_ucy_loo_kfold4 eth_ucy_real || exit 1 ;;
overhead) bash tools/gpu_overhead.sh ${TAG}_ov || exit 1 ;;
esac
done
