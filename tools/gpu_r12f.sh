# r12f: train-mode workgroup timeline (eth_hotel_synth, kfold4; one launch at a time)
set -o pipefail
O=gpurun_out/r12f; mkdir -p $O
TL_TRAIN=1 TL_OUT=tools/ab/tl_peel.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 1 0 > $O/tl_train_eth1.txt 2>&1 &&
TL_TRAIN=1 TL_OUT=tools/ab/tl_peel.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_ucy_loo_kfold4 1 0 > $O/tl_train_kf1.txt 2>&1
