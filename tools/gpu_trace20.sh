#!/bin/bash
# kernel trace of the driver's invocation (20 steps) for the replay span
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { echo "trace failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | cut -c1-200
python tools/trace_span.py $O/trace 20
