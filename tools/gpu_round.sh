#!/bin/bash
# One GPU session: tests, smoke, bench under rocprof (kernel trace + stats),
# PMC traffic passes (reference mode and train mode), 1-GPU bench lines of the
# other configs.  Every GPU step has its own time limit; stops at the first
# failure.  Outputs under gpurun_out/$TAG.
set -o pipefail
TAG=${1:-r2}
CFG=${2:-eth_hotel_synth}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
grep smoke: $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config $CFG > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-400
python tools/pmc_summary.py $O/trace
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -5 $O/pmc_write.log; exit 1; }
python tools/collect_pmc.py $O/pmc_fetch $O/pmc_write $CFG $O/pmc_$CFG.json ref
python tools/collect_pmc.py $O/pmc_fetch $O/pmc_write ${CFG}_train $O/pmc_${CFG}_train.json train
for c in eth_ucy_loo_kfold4 relational_attn_h256 dense_crowd; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 100 > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -10 $O/bench_$c.log; exit 1; }
  grep '^{' $O/bench_$c.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"], "fwd us", round(d["ms_per_step"]*1e3,2), "train us", round(d["train_mode"]["ms_per_step"]*1e3,2))'
done
