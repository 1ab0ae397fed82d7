# r12g: timing probe — train with every frame reading frame 0's targets (cache-resident) vs the peeled tree
set -o pipefail
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12g 2 "tools/ab/peel.so tools/ab/tfb0.so" eth_hotel_synth eth_ucy_loo_kfold4
