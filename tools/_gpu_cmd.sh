set -o pipefail
O=gpurun_out/${1:-d39}; mkdir -p $O
export TMPDIR=/tmp
b() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-train --steps 400 "${EXTRA[@]}" > $O/bench_$lab.log 2>&1 || { tail -20 $O/bench_$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/bench_$lab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), "us/step", round(d["roofline"]["kernel_us"],2), "us kernel")')"
}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
EXTRA=(--config eth_ucy_loo_kfold4)
b kf8 G2K_SCENE_NP=8 && b kf12 G2K_SCENE_NP=12
EXTRA=()
b default
EXTRA=(--config relational_attn_h256)
b h256default
