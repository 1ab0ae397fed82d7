#!/bin/bash
# A/B of the fused scene kernel against the two-kernel split step (G2K_STEP_SPLIT=1)
# and the producer-wave counts; one bench line each (no CPU baseline).
set -o pipefail
O=gpurun_out/${1:-ab}
CFG=${2:-eth_hotel_synth}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for np in 8 4; do
  G2K_SCENE_NP=$np timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline > $O/bench_np$np.log 2>&1 || { echo "bench np$np failed"; tail -20 $O/bench_np$np.log; exit 1; }
  echo "np=$np $(grep '^{' $O/bench_np$np.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_us"])')"
done
G2K_STEP_SPLIT=1 timeout -k 10 120 python bench.py --config $CFG --no-cpu-baseline > $O/bench_split.log 2>&1 || { echo "bench split failed"; tail -20 $O/bench_split.log; exit 1; }
echo "split $(grep '^{' $O/bench_split.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_us"])')"
