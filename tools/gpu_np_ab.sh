# Producer-count A/B (G2K_SCENE_NP 12 vs 4: one 16-wave workgroup per CU vs two
# co-resident 8-wave ones), interleaved bench lines per config and stream count.
#   tools/gpu_np_ab.sh TAG ROUNDS CONFIG...
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $R); do
for c in "$@"; do
for st in 2 3; do
for np in 12 4; do
  G2K_SCENE_NP=$np timeout -k 10 120 python bench.py --no-cpu-baseline --no-train --config $c --streams $st --steps 400 > $O/b_${c}_${np}_${st}_$r.txt 2>&1 || { echo "bench $c np $np failed"; tail -20 $O/b_${c}_${np}_${st}_$r.txt; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; print(sys.argv[2], 'us/step %.2f launch %.2f frac %.3f' % (d['ms_per_step']*1e3, r['kernel_us'], r['frac']))" $O/b_${c}_${np}_${st}_$r.txt "$c np=$np streams=$st"
done; done; done; done
