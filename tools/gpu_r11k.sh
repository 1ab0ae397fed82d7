set -o pipefail
O=gpurun_out/r11k; mkdir -p $O
for st in 4 6 8; do
AB_ARGS="--streams $st" bash tools/gpu_lib_ab.sh r11k_s$st 1 "tree tools/ab/inv4.so" eth_ucy_real | sed "s/^/streams $st: /"
done
