#!/bin/bash
# Round 6 first session: the RCCL capture tests (no sleep, reap before
# capture), the default bench (flop roofline), the collective bench captured.
set -o pipefail
O=gpurun_out/r10a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py tests/test_split_gpu.py tests/test_abi.py -x -v --timeout 240 --timeout-method thread > $O/rccl.log 2>&1 || { echo "rccl tests failed"; tail -60 $O/rccl.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/rccl.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -30 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
timeout -k 10 300 python bench.py --collective on --no-cpu-baseline --steps 20 --warmup 5 > $O/bench_coll.log 2>&1 || { echo "bench coll failed"; tail -30 $O/bench_coll.log; exit 1; }
grep '^{' $O/bench_coll.log > $O/bench_coll.json
python - <<'PY'
import json
for f in ("gpurun_out/r10a/bench.json", "gpurun_out/r10a/bench_coll.json"):
    d = json.load(open(f)); r = d["roofline"]; t = d["train_mode"]
    print(f, "us/step %.2f" % (d["ms_per_step"]*1e3), {k: r[k] for k in ("bound","achieved","unit","frac","intensity","frac_hbm","frac_flops","frac_hbm_per_step","frac_flops_per_step","kernel_us")})
    print("  train", "%.2f us" % (t["ms_per_step"]*1e3), t["step_structure"], t.get("collective_parts_us"), {k: t["roofline"][k] for k in ("bound","frac","intensity","frac_hbm","frac_flops")})
PY
