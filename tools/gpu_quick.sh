# quick GPU session: the GPU tests, the launch probe, the headline bench with
# and without graph replay.   tools/gpu_quick.sh TAG
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 5 120 python tools/probes/launch_probe.py > $O/launch.txt 2>&1 || { echo "launch probe failed"; tail -20 $O/launch.txt; exit 1; }
grep -v amdgpu.ids $O/launch.txt
for g in "" "--no-graph"; do
timeout -k 10 200 python bench.py --no-cpu-baseline $g > $O/bench$g.txt 2>&1 || { echo "bench $g failed"; tail -20 $O/bench$g.txt; exit 1; }
python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; r=d['roofline']; t=d['train_mode']; print(sys.argv[2] or 'graph', 'fwd us %.2f kern %.2f frac %.3f | train us %.2f step %.2f' % (d['ms_per_step']*1e3, r['kernel_us'], r['frac'], t['ms_per_step']*1e3, t['roofline']['step_us']))" $O/bench$g.txt "$g"
done
