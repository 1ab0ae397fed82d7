# loop-invariant train path: GPU tests (layouts, real data, train, split, train mode), then real-data train A/B vs HEAD
set -o pipefail
O=gpurun_out/r11r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_layouts_gpu.py tests/test_realdata_gpu.py tests/test_train_gpu.py tests/test_split_gpu.py tests/test_train_mode_gpu.py tests/test_train_nll_gpu.py tests/test_rccl_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r11r 2 "tree tools/ab/head.so" eth_ucy_real eth_hotel_synth
