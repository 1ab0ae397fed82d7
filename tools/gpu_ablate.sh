# ablation timings of the scene kernel (tools/ab_time.py variants)
set -o pipefail
O=gpurun_out/abl; mkdir -p $O
for c in eth_hotel_synth; do
timeout -k 10 300 python tools/ab_time.py --rounds 3 $c base no_tile_mfma no_m_mfma no_tiles no_recur > $O/abl2_$c.log 2>&1 || { echo "abl failed"; tail -20 $O/abl2_$c.log; exit 1; }
grep median $O/abl2_$c.log
done
