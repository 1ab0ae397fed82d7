# r12j: train finalize — producer 0's dWi tile run twice (first run vs warm code), eth_hotel_synth and kfold4, one launch at a time
set -o pipefail
O=gpurun_out/r12j; mkdir -p $O
TL_TRAIN=1 TL_OUT=tools/ab/tl_dwi.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 1 0 > $O/tl_eth.txt 2>&1 &&
TL_TRAIN=1 TL_OUT=tools/ab/tl_dwi.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_ucy_loo_kfold4 1 0 > $O/tl_kf.txt 2>&1
