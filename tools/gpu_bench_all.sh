# the headline bench under rocprofv3 (kernel trace + stats) and one bench line
# per config (reading the committed PMC summaries).   tools/gpu_bench_all.sh TAG
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
python tools/pmc_summary.py $O/trace | grep -E "g2k_"
for c in eth_hotel_synth eth_ucy_loo_kfold4 relational_attn_h256 dense_crowd eth_ucy_real; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 200 > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -10 $O/bench_$c.log; exit 1; }
  grep '^{' $O/bench_$c.log > $O/bench_$c.json
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; t=d["train_mode"]; print(d["config"]["workload"], "fwd us %.2f kern %.2f frac %.3f traffic/alg %.2f | train us %.2f frac %.3f" % (d["ms_per_step"]*1e3, r["kernel_us"], r["frac"], (r["traffic"] or 0)/r["algorithmic_bytes"], t["ms_per_step"]*1e3, t["roofline"]["frac"]))' $O/bench_$c.json
done
