# rocprof kernel stats of the train step's tail (tools/probes/train_tail.py)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/probes/train_tail.py > $O/tail.log 2>&1 || { echo "tail failed"; tail -20 $O/tail.log; exit 1; }
f=$(ls $O/trace/*/*kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] || f=$(ls $O/trace/*kernel_stats.csv | head -1)
cut -c1-220 $f
