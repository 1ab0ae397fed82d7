# r12b: lead priority (s_setprio 3 from entry / from B1 to the first B2) A/B, forward
set -o pipefail
bash tools/gpu_lib_ab.sh r12b 2 "tools/ab/base.so tools/ab/lp1.so tools/ab/lp2.so" eth_hotel_synth eth_ucy_loo_kfold4 eth_ucy_real
