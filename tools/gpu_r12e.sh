# r12e: the first staging task peeled out of the task loop (forward kernels): timeline, A/B (400 steps), driver's invocation
set -o pipefail
O=gpurun_out/r12e; mkdir -p $O
TL_OUT=tools/ab/tl_peel.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 1 0 on > $O/tl_eth1.txt 2>&1 &&
TL_OUT=tools/ab/tl_peel.so timeout -k 10 180 python tools/probes/wg_timeline.py eth_hotel_synth 16 0 on > $O/tl_eth16.txt 2>&1 &&
grep -h "vtile\|lead" $O/tl_eth1.txt $O/tl_eth16.txt &&
bash tools/gpu_lib_ab.sh r12e 2 "tools/ab/base.so tools/ab/peel.so" eth_hotel_synth eth_ucy_loo_kfold4 eth_ucy_real dense_crowd relational_attn_h256 &&
for r in 1 2 3 4; do for l in base peel; do
  timeout -k 10 120 python tools/bench_lib.py tools/ab/$l.so --steps 20 --warmup 5 --no-cpu-baseline --no-train > $O/d_${l}_$r.log 2>&1 || { echo fail; tail -5 $O/d_${l}_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('driver', sys.argv[2], 'r', sys.argv[3], 'us/step %.2f' % (d['ms_per_step']*1e3))" $O/d_${l}_$r.log $l $r
done; done
