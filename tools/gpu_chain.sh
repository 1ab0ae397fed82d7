#!/bin/bash
# --use_grid_lstm chain: the GPU tests (bit-identity vs the three-launch
# loop, per-frame time) and a rocprofv3 kernel trace of the timing test.
#   tools/gpu_chain.sh TAG
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_encoder_chain_gpu.py -v -s --timeout 120 --timeout-method thread > $O/chain.log 2>&1 || { echo "chain tests failed"; tail -40 $O/chain.log; exit 1; }
grep -E "PASSED|FAILED|us_per_frame" $O/chain.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 -m pytest tests/test_encoder_chain_gpu.py::test_chain_entry_time_per_frame -q > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/trace -name '*kernel_stats.csv' | head -1); cp $f $O/chain_kernel_stats.csv; cut -d, -f1-8 $f | head -12
