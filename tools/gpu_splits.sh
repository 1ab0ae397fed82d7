set -o pipefail
O=gpurun_out/splits; mkdir -p $O
for c in dense_crowd eth_ucy_loo_kfold4; do
 for x in 2 3 4; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 100 --split $x > $O/b_${c}_$x.log 2>&1 || { echo "bench $c $x failed"; tail -20 $O/b_${c}_$x.log; exit 1; }
  python -c 'import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]; r=d["roofline"]; t=d["train_mode"]; print(sys.argv[2], sys.argv[3], "fwd us %.2f kern %.2f | train us %.2f" % (d["ms_per_step"]*1e3, r["kernel_us"], t["ms_per_step"]*1e3))' $O/b_${c}_$x.log $c $x
 done
done
