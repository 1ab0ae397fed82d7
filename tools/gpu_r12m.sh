# r12m: block ownership (workgroup 0 = one frame per producer) + free recurrence waves in the chain-less workgroup = the tree: GPU tests, then train A/B vs HEAD (peel) on every config
set -o pipefail
O=gpurun_out/r12m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_train_mode_gpu.py tests/test_layouts_gpu.py tests/test_split_gpu.py tests/test_realdata_gpu.py tests/test_train_nll_gpu.py tests/test_step_gpu.py tests/test_rccl_gpu.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12m 2 "tools/ab/peel.so tools/ab/own8.so" eth_ucy_loo_kfold4 eth_hotel_synth relational_attn_h256 dense_crowd eth_ucy_real
