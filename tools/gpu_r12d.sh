# r12d: producer 0's first V tile, stamped (one launch at a time; 16 streams)
set -o pipefail
O=gpurun_out/r12d; mkdir -p $O
TL_OUT=tools/ab/tl_vtile.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 1 0 on > $O/tl_eth1.txt 2>&1 &&
TL_OUT=tools/ab/tl_vtile.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 16 0 on > $O/tl_eth16.txt 2>&1
