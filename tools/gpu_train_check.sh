#!/bin/bash
# train-mode GPU tests, then an interleaved A/B of the train line against a
# previous build.   tools/gpu_train_check.sh TAG PREV_LIB [CONFIG...]
set -o pipefail
TAG=$1; PREV=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_split_gpu.py tests/test_train_nll_gpu.py tests/test_train_mode_gpu.py tests/test_train_legs_gpu.py -v -m gpu --maxfail=3 --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || { echo "pytest rc $rc"; exit 1; }
AB_TRAIN=1 tools/gpu_lib_ab.sh $TAG 3 "tree $PREV" "$@"
