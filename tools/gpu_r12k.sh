# r12k: block frame ownership for two-workgroup train scenes (workgroup 0 owns own0/256 of each chunk): GPU tests (tree = 90), then kfold4 train A/B vs HEAD (modular)
set -o pipefail
O=gpurun_out/r12k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_train_mode_gpu.py tests/test_layouts_gpu.py tests/test_split_gpu.py tests/test_realdata_gpu.py tests/test_train_nll_gpu.py tests/test_step_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12k 3 "tools/ab/peel.so tools/ab/own77.so tools/ab/own90.so tools/ab/own102.so" eth_ucy_loo_kfold4
