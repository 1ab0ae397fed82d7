# Interleaved A/B of library builds on bench lines (400 steps; coresident,
# 4 streams): tools/gpu_lib_ab.sh TAG ROUNDS "LIB..." CONFIG...
# (LIB "tree" = the in-tree libg2k_hip.so; AB_TRAIN=1: also time train mode)
set -o pipefail
TAG=$1; R=$2; LIBS=$3; shift 3
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $R); do
for c in "$@"; do
for l in $LIBS; do
  p=$l; [ $l = tree ] && p=multimodaltraj_2_amd/libg2k_hip.so
  f=$O/b_${c}_$(basename $l .so)_$r.txt
  timeout -k 10 120 python tools/bench_lib.py $p --no-cpu-baseline $([ -z "$AB_TRAIN" ] && echo --no-train) --config $c --steps 400 ${AB_ARGS} > $f 2>&1 || { echo "bench $c $l failed"; tail -20 $f; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; t=d.get('train_mode'); print(sys.argv[2], 'us/step %.2f launch %.2f' % (d['ms_per_step']*1e3, r['kernel_us']), ('train us/step %.2f' % (t['ms_per_step']*1e3)) if t else '')" $f "$c $(basename $l .so) r$r"
done; done; done
