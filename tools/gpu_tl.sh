# Workgroup timelines (tools/probes/wg_timeline.py, prebuilt tools/ab/libg2k_timeline.so):
# each spec CONFIG:CORES:STREAMS:SPLIT (CORES on|off).   tools/gpu_tl.sh TAG SPEC...
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for spec in "$@"; do
  IFS=: read c co st sp <<< "$spec"
  timeout -k 10 120 python tools/probes/wg_timeline.py $c $st $sp $co > $O/tl_${c}_${co}_${st}_${sp}.txt 2>&1 || { echo "timeline $spec failed"; tail -20 $O/tl_${c}_${co}_${st}_${sp}.txt; exit 1; }
  grep -v amdgpu.ids $O/tl_${c}_${co}_${st}_${sp}.txt
done
