set -o pipefail
O=gpurun_out/r11e; mkdir -p $O
timeout -k 10 120 python tools/probes/chain_stamps.py tools/ab/chain_stamps.so > $O/stamps.txt 2>&1 || { echo stamps failed; tail -20 $O/stamps.txt; exit 1; }
grep "^H" $O/stamps.txt
timeout -k 10 500 python -u -m pytest tests/test_encoder_chain_gpu.py tests/test_gridlstm.py tests/test_train_legs_gpu.py tests/test_models_gpu.py tests/test_sample_gpu.py tests/test_layouts_gpu.py tests/test_step_gpu.py -v -s --timeout 120 --timeout-method thread > $O/chain.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/chain.log | head -30; tail -30 $O/chain.log; exit 1; }
grep -E "PASSED|FAILED|us_per_frame" $O/chain.log
