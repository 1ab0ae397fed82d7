# A/B at 16 streams: tree vs np2 (three 6-wave co-resident workgroups per CU: 2 producers, <= 96 VGPRs, the window aliased onto the rings)
set -o pipefail
bash tools/gpu_lib_ab.sh r11o 2 "tree tools/ab/np2.so" eth_hotel_synth eth_ucy_real relational_attn_h256
