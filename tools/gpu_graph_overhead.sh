# Fixed cost of a short timed region (tools/probes/graph_overhead.py):
# rounds of {default, upload, prereplay} at --steps K.   tools/gpu_graph_overhead.sh TAG ROUNDS K
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for r in $(seq $2); do
for m in ${MODES:-default upload prereplay}; do
  f=$O/g_${m}_$r.txt
  timeout -k 10 120 python tools/probes/graph_overhead.py $m $3 > $f 2>&1 || { echo "$m failed"; tail -20 $f; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(sys.argv[2], 'us/step %.2f' % (d['ms_per_step']*1e3))" $f "$m K=$3 r$r"
done; done
