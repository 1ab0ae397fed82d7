# r12l: kfold4 train — block ownership fractions and free recurrence waves in the chain-less workgroup (rf)
set -o pipefail
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12l 2 "tools/ab/peel.so tools/ab/own102.so tools/ab/own115.so tools/ab/own102rf.so tools/ab/own90rf.so tools/ab/own0rf.so" eth_ucy_loo_kfold4
