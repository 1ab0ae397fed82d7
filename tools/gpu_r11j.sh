# loop-invariant frames (stride 0, shared targets): GPU tests, then A/B vs HEAD's build
set -o pipefail
O=gpurun_out/r11j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_layouts_gpu.py tests/test_realdata_gpu.py tests/test_step_gpu.py tests/test_split_gpu.py tests/test_sample_gpu.py tests/test_train_legs_gpu.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_lib_ab.sh r11j 2 "tree tools/ab/inv4.so tools/ab/base.so" eth_ucy_real
