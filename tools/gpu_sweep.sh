# Bench sweep over launch geometries: each spec is CONFIG:CORES:SPLIT:STREAMS
# (CORES = --coresident on|off, SPLIT = --split, 0 automatic), R interleaved rounds.
#   tools/gpu_sweep.sh TAG R SPEC...
set -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
for r in $(seq $R); do
for spec in "$@"; do
  IFS=: read c co sp st <<< "$spec"
  f=$O/b_${c}_${co}_${sp}_${st}_$r.txt
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-train --config $c --coresident $co --split $sp --streams $st --steps 400 > $f 2>&1 || { echo "bench $spec failed"; tail -20 $f; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; print(sys.argv[2], 'X=%d us/step %.2f launch %.2f' % (d['config']['workgroups_per_scene'], d['ms_per_step']*1e3, r['kernel_us']))" $f "$spec r$r"
done; done
