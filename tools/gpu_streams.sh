# reference-mode batches on 1 or 2 streams (graph replay)
set -o pipefail
O=gpurun_out/streams; mkdir -p $O
for c in eth_hotel_synth eth_ucy_loo_kfold4; do
 for n in 1 2; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-train --streams $n > $O/b_${c}_$n.log 2>&1 || { echo "bench $c $n failed"; tail -20 $O/b_${c}_$n.log; exit 1; }
  python -c 'import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]; r=d["roofline"]; print(sys.argv[2], sys.argv[3], "fwd us %.2f kern %.2f frac %.3f" % (d["ms_per_step"]*1e3, r["kernel_us"], r["frac"]))' $O/b_${c}_$n.log $c $n
 done
done
