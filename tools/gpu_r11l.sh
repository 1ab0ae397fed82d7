# invariant path (4 producers, one-slot rings): GPU tests; streams 4 vs 8 per config
set -o pipefail
O=gpurun_out/r11l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_layouts_gpu.py tests/test_realdata_gpu.py tests/test_sample_gpu.py tests/test_train_legs_gpu.py -x -v --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/tests.log | head -20; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for st in 4 8; do
AB_ARGS="--streams $st" bash tools/gpu_lib_ab.sh r11l_s$st 1 "tree" eth_ucy_real eth_ucy_loo_kfold4 dense_crowd eth_hotel_synth relational_attn_h256 | sed "s/^/streams $st: /"
done
