# attn_weights exchanges / row softmax + tile el2: GPU tests of the step, then A/B vs HEAD's build
set -o pipefail
O=gpurun_out/r11h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_step_gpu.py tests/test_split_gpu.py tests/test_train_gpu.py tests/test_errors_gpu.py tests/test_realdata_gpu.py tests/test_layouts_gpu.py -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r11h 2 "tree tools/ab/base.so" eth_hotel_synth eth_ucy_loo_kfold4 eth_ucy_real
