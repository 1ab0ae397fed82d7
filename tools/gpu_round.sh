#!/bin/bash
# One GPU session: tests, smoke, bench under rocprof (kernel trace + stats),
# PMC traffic passes, 1-GPU bench lines of the other configs.  Every GPU step
# has its own time limit; stops at the first failure.  Outputs under
# gpurun_out/$TAG.
set -o pipefail
TAG=${1:-r1}
CFG=${2:-eth_hotel_synth}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
grep smoke: $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config $CFG > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-300
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-train > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --no-cpu-baseline --no-train > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -5 $O/pmc_write.log; exit 1; }
python tools/collect_pmc.py $O/pmc_fetch $O/pmc_write $CFG $O/pmc_$CFG.json
python tools/pmc_summary.py $O/trace
for c in eth_ucy_loo_kfold4 relational_attn_h256 dense_crowd; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 100 > $O/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -10 $O/bench_$c.log; exit 1; }
  grep '^{' $O/bench_$c.log | cut -c1-160
done
