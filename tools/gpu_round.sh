#!/bin/bash
# One GPU session: tests, smoke, the headline bench under rocprof (kernel
# trace + stats), PMC traffic passes for EVERY config (FETCH_SIZE, WRITE_SIZE:
# separate runs; reference and train mode from the same passes), then one
# bench line per config reading the fresh PMC.  Every GPU step has its own
# time limit; stops at the first failure.  Outputs under gpurun_out/$TAG
# (the PMC summaries are also copied into profiles/ on the box, where the
# bench lines read them).
#   tools/gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-r3}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
  grep smoke: $O/smoke.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300
python tools/pmc_summary.py $O/trace
for c in eth_hotel_synth eth_ucy_loo_kfold4 relational_attn_h256 dense_crowd eth_ucy_real; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_fetch_$c.log 2>&1 || { echo "pmc fetch $c failed"; tail -5 $O/pmc_fetch_$c.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$c -o run -- python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_write_$c.log 2>&1 || { echo "pmc write $c failed"; tail -5 $O/pmc_write_$c.log; exit 1; }
  python tools/collect_pmc.py $O/pmc_fetch_$c $O/pmc_write_$c $c $O/pmc_$c.json ref > /dev/null
  python tools/collect_pmc.py $O/pmc_fetch_$c $O/pmc_write_$c ${c}_train $O/pmc_${c}_train.json train > /dev/null
  cp $O/pmc_$c.json profiles/pmc_$c.json && cp $O/pmc_${c}_train.json profiles/pmc_${c}_train.json
  rm -rf $O/pmc_fetch_$c $O/pmc_write_$c
done
for c in eth_hotel_synth eth_ucy_loo_kfold4 relational_attn_h256 dense_crowd eth_ucy_real; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 200 > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -10 $O/bench_$c.log; exit 1; }
  grep '^{' $O/bench_$c.log > $O/bench_$c.json
  python -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; t=d["train_mode"]; print(d["config"]["workload"], "fwd us %.2f kern %.2f frac %.3f traffic/alg %.2f | train us %.2f frac %.3f" % (d["ms_per_step"]*1e3, r["kernel_us"], r["frac"], (r["traffic"] or 0)/r["algorithmic_bytes"], t["ms_per_step"]*1e3, t["roofline"]["frac"]))' $O/bench_$c.json
done
