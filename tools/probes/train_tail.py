"""train_tail — the train step's tail kernels at eth_hotel_synth's shape, for
rocprofv3 --kernel-trace --stats: the fused row sum + update
(g2k_grad_rows_kernel<true>), the row sum alone (<false>) and the separate
update (g2k_update_kernel).  Development probe (timing only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from multimodaltraj_2_amd import frame_step as fs, train_step as ts  # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "eth_hotel_synth"
c = CONFIGS[cfg]
S = c["S"] if c["S"] <= 256 else c["S"] // 8
dev = torch.device("cuda")
t = make_batch(S, c["Nmax"], c["H"], seed=1).to_device(dev)
params = fs.init_params(c["Nmax"], seed=0, device=dev)
keys = ("pos", "vislet", "G", "targets", "n_active", "h0")
step = ts.TrainStep(params, *(t[k] for k in keys))
tp = ts.TrainPlan(params, *(t[k] for k in keys))
flat, _ = ts.flat_params(params)
ms = torch.ones_like(flat)
for _ in range(200):
    step.run()
for _ in range(200):
    g = tp.run()
    ts.optimizer_update(flat, g, ms=ms)
torch.cuda.synchronize()
print("done", cfg, S)
