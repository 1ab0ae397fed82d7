# r12p: the own-frame stride as an inline expression (the INV train kernel's SGPR spills back to 162) = blk2 vs blk (r12n) vs HEAD~ (peel): train A/B
set -o pipefail
O=gpurun_out/r12p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_split_gpu.py tests/test_realdata_gpu.py tests/test_layouts_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12p 2 "tools/ab/peel.so tools/ab/blk.so tools/ab/blk2.so" eth_ucy_real eth_ucy_loo_kfold4 eth_hotel_synth
