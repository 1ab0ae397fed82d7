# r12v: the chain-less workgroup's recurrence waves take cnt - NP frames when fewer than four are left over (rfr) vs the tree (blk5): dense_crowd (11 frames on workgroup 1), kfold4; split tests with rfr in-tree first
set -o pipefail
O=gpurun_out/r12v; mkdir -p $O
timeout -k 10 150 python -u -m pytest tests/test_split_gpu.py tests/test_train_gpu.py -x -q --timeout 100 --timeout-method thread > $O/split.log 2>&1 || { echo "tests failed"; tail -30 $O/split.log; exit 1; }
tail -1 $O/split.log
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12v 2 "tools/ab/blk5.so tools/ab/rfr.so" dense_crowd eth_ucy_loo_kfold4
