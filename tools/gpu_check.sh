#!/bin/bash
# GPU check: the GPU test suite (at most 5 failures), smoke, the default
# bench line.   tools/gpu_check.sh TAG [pytest selection...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
SEL=${@:-tests}
timeout -k 10 900 python -u -m pytest $SEL -v -m gpu --maxfail=5 --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -eq 0 ] || { echo "pytest rc $rc"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
grep smoke: $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; t=d['train_mode']; print('fwd us %.2f kern %.2f frac %.3f | train us %.2f' % (d['ms_per_step']*1e3, r['kernel_us'], r['frac'], t['ms_per_step']*1e3))" $O/bench.log
