# r12r: block ownership also for frame-ordered dWo (dense_crowd's split scenes) = blk3: the split tests first under a short limit (a wrong frame ordinal would spin), then train tests, then train A/B vs blk2 (HEAD)
set -o pipefail
O=gpurun_out/r12r; mkdir -p $O
timeout -k 10 150 python -u -m pytest tests/test_split_gpu.py -x -v --timeout 100 --timeout-method thread > $O/split.log 2>&1 || { echo "split tests failed"; tail -30 $O/split.log; exit 1; }
tail -1 $O/split.log
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_train_mode_gpu.py tests/test_layouts_gpu.py tests/test_realdata_gpu.py tests/test_train_nll_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12r 2 "tools/ab/blk2.so tools/ab/blk3.so" dense_crowd eth_ucy_loo_kfold4
