#!/bin/bash
# Timeline A/B: each prebuilt probe library (tools/ab/libg2k_tl_<v>.so) on the
# same specs.   tools/gpu_tl_ab.sh TAG "v1 v2 ..." SPEC...   (SPEC CONFIG:CORES:STREAMS:SPLIT[:train])
set -o pipefail
O=gpurun_out/$1; VS=$2; shift 2; mkdir -p $O
for spec in "$@"; do
  IFS=: read c co st sp tr <<< "$spec"
  for v in $VS; do
    f=$O/tl_${v}_${c}_${co}_${st}_${sp}_${tr}.txt
    if [ "$tr" = train ]; then export TL_TRAIN=1; else unset TL_TRAIN; fi
    TL_OUT=tools/ab/libg2k_tl_$v.so timeout -k 10 120 python tools/probes/wg_timeline.py $c $st $sp $co > $f 2>&1 || { echo "timeline $v $spec failed"; tail -20 $f; exit 1; }
    echo "== $v $spec"; grep -v amdgpu.ids $f | grep -v "^launch"
  done
done
