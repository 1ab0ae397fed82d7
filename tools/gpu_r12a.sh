# r12a: workgroup timelines of the final tree (eth_hotel_synth coresident: 16 streams and one
# launch at a time; eth_ucy_real-like lone launch is not covered by the probe)
set -o pipefail
O=gpurun_out/r12a; mkdir -p $O
timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 16 0 on > $O/tl_eth16.txt 2>&1 &&
timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 1 0 on > $O/tl_eth1.txt 2>&1 &&
timeout -k 10 180 python tools/probes/wg_timeline.py eth_ucy_loo_kfold4 16 0 on > $O/tl_kf16.txt 2>&1
