#!/bin/bash
# gradient kernel: GPU train tests, then tools/diag_grad.py at two configs
set -o pipefail
O=gpurun_out/${1:-grad}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in eth_hotel_synth dense_crowd; do
  timeout -k 10 200 python tools/diag_grad.py $c > $O/diag_$c.log 2>&1 || { tail -20 $O/diag_$c.log; exit 1; }
  grep -v amdgpu.ids $O/diag_$c.log
done
