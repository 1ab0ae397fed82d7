"""Run the reference-mode step alone (profiling driver, not product code):
python tools/fwd_only.py [CONFIG] [REPS]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import frame_step as fs  # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "eth_hotel_synth"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
c = CONFIGS[cfg]
S = c["S"] if c["S"] <= 256 else c["S"] // 8
dev = torch.device("cuda")
t = make_batch(S, c["Nmax"], c["H"], seed=1).to_device(dev)
params = fs.init_params(c["Nmax"], seed=0, device=dev)
plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
for _ in range(reps):
    plan.run()
torch.cuda.synchronize()
print("done", cfg, reps)
