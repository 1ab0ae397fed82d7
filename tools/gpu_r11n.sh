# 16 streams: co-resident geometry on vs off (400 steps), and the driver's invocation
set -o pipefail
O=gpurun_out/r11n; mkdir -p $O
for c in eth_hotel_synth eth_ucy_loo_kfold4 relational_attn_h256; do for co in on off; do
  timeout -k 10 120 python bench.py --config $c --steps 400 --no-cpu-baseline --no-train --coresident $co > $O/${c}_$co.log 2>&1 || { echo fail; tail -5 $O/${c}_$co.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print(d['config']['workload'], 'coresident', d['config']['coresident'], 'streams', d['config']['streams'], 'us/step %.2f launch %.2f' % (d['ms_per_step']*1e3, d['roofline']['kernel_us']))" $O/${c}_$co.log
done; done
for r in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-train > $O/drv_$r.log 2>&1 || { echo fail; tail -5 $O/drv_$r.log; exit 1; }
  python -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][0]; print('driver-like', 'us/step %.2f value %.3e' % (d['ms_per_step']*1e3, d['value']))" $O/drv_$r.log
done
