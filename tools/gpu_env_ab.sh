# A/B of one runtime environment variable on bench lines (coresident, 4
# streams): tools/gpu_env_ab.sh TAG ROUNDS VAR "VALUES" STEPS CONFIG...
set -o pipefail
TAG=$1; R=$2; VAR=$3; VALS=$4; STEPS=$5; shift 5
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $R); do
for c in "$@"; do
for v in $VALS; do
  f=$O/b_${c}_${VAR}_${v}_$r.txt
  if [ "$v" = unset ]; then E="env -u $VAR"; else E="env $VAR=$v"; fi   # unset: the runtime's default
  $E timeout -k 10 120 python bench.py --no-cpu-baseline --no-train --config $c --steps $STEPS --warmup 5 > $f 2>&1 || { echo "bench $c $VAR=$v failed"; tail -20 $f; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; print(sys.argv[2], 'us/step %.2f launch %.2f' % (d['ms_per_step']*1e3, r['kernel_us']))" $f "$c $VAR=$v steps=$STEPS r$r"
done; done; done
