set -o pipefail
O=gpurun_out/s1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for c in eth_ucy_loo_kfold4 dense_crowd eth_ucy_real eth_hotel_synth; do
 for x in 1 0; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 200 --split $x > $O/b_${c}_$x.log 2>&1 || { echo "bench $c $x failed"; tail -20 $O/b_${c}_$x.log; exit 1; }
  python -c 'import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][0]; r=d["roofline"]; t=d["train_mode"]; print(sys.argv[2], sys.argv[3], "fwd us %.2f kern %.2f | train us %.2f" % (d["ms_per_step"]*1e3, r["kernel_us"], t["ms_per_step"]*1e3))' $O/b_${c}_$x.log $c $x
 done
done
