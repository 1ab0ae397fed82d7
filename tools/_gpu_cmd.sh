set -o pipefail
O=gpurun_out/${1:-d29}; mkdir -p $O
export TMPDIR=/tmp
b() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps 400 > $O/bench_$lab.log 2>&1 || { tail -20 $O/bench_$lab.log; return 1; }
  echo "$lab $(grep '^{' $O/bench_$lab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"]*1e3,2), "us/step", round(d["roofline"]["kernel_us"],2), "us kernel")')"
}
timeout -k 10 300 python -u -m pytest tests/test_step_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
b ae31 G2K_LIB_PATH=tools/ab/lib_ae31.so && b o0 G2K_SCENE_OPTS=0 && b o1 G2K_SCENE_OPTS=1 && b o2 G2K_SCENE_OPTS=2 && b o3 G2K_SCENE_OPTS=3 && b o0nodma G2K_SCENE_OPTS=0 G2K_NO_DMA16=1 && b ae31b G2K_LIB_PATH=tools/ab/lib_ae31.so
