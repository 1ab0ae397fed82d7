set -o pipefail
O=gpurun_out/r11d; mkdir -p $O
timeout -k 10 120 python tools/probes/chain_stamps.py tools/ab/chain_stamps.so > $O/stamps.txt 2>&1 || { echo stamps failed; tail -20 $O/stamps.txt; exit 1; }
grep "^H" $O/stamps.txt
bash tools/gpu_lib_ab.sh r11d 2 "tree tools/ab/cr3.so" eth_hotel_synth eth_ucy_loo_kfold4 eth_ucy_real
