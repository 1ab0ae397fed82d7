# r12c: lead priority at the driver's invocation (20 steps, warm-up 5), four interleaved rounds;
# then train mode (400 steps) and dense_crowd forward
set -o pipefail
O=gpurun_out/r12c; mkdir -p $O
for r in 1 2 3 4; do for l in base lp1 lp2; do
  timeout -k 10 120 python tools/bench_lib.py tools/ab/$l.so --steps 20 --warmup 5 --no-cpu-baseline --no-train > $O/d_${l}_$r.log 2>&1 || { echo fail; tail -5 $O/d_${l}_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('driver', sys.argv[2], 'r', sys.argv[3], 'us/step %.2f' % (d['ms_per_step']*1e3))" $O/d_${l}_$r.log $l $r
done; done
AB_TRAIN=1 bash tools/gpu_lib_ab.sh r12c 2 "tools/ab/base.so tools/ab/lp1.so tools/ab/lp2.so" eth_hotel_synth dense_crowd
