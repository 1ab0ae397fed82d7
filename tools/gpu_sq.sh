#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per group, 8 SQ counters each)
# over the default bench (co-resident forward on 4 streams + train mode).
#   tools/gpu_sq.sh TAG [bench args...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SMEM"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python tools/pmc_sq.py $O/p1 $O/p2 | tee $O/sq_summary.txt
