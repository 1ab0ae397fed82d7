# r12s: dense_crowd split scenes with block ownership at fc/2 - 1 frames for workgroup 0 (blk4) vs the tree (blk2, modular there); split tests with blk4 loaded first
set -o pipefail
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12s 2 "tools/ab/blk2.so tools/ab/blk4.so" dense_crowd
