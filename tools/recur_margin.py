"""Measured error of the fused step's split-f16 recurrence product against the
float64 oracle (development record for DESIGN.md "Recurrence numerics"):
worst |dh| / (|h| + 1e-3 / H) over every entry of h after F frames, per H,
from zero and from N(0, 1) initial states.

usage: python tools/recur_margin.py [F] [S]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import frame_step as fs  # noqa: E402
from multimodaltraj_2_amd.synthetic import make_batch  # noqa: E402
from oracle import g2k_ref as ref  # noqa: E402

F = int(sys.argv[1]) if len(sys.argv) > 1 else 100
S = int(sys.argv[2]) if len(sys.argv) > 2 else 4
dev = torch.device("cuda")
print(f"# split-f16 recurrence vs float64 oracle: S={S} scenes, Nmax 32, F={F} frames; "
      "worst |dh|/(|h| + 1e-3/H) and worst |dh|/|h| over entries with |h| > 1e-3/H")
for H in (64, 128, 256, 512):
    for h0 in (0.0, 1.0):
        b = make_batch(S, 32, H, F=F, seed=7, h0_scale=h0)
        t = b.to_device(dev)
        p = fs.init_params(32, seed=0, device=dev)
        out = fs.step_fused(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
        torch.cuda.synchronize()
        hh = out.h.cpu().numpy().astype(np.float64)
        w = p.numpy()
        worst = worst_rel = 0.0
        for s in range(S):
            _, h, _, _ = ref.scene_step(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s], b.n_active[s],
                                        b.h0[s], n_frames=F)
            d = np.abs(hh[s] - h)
            worst = max(worst, float(np.max(d / (np.abs(h) + 1e-3 / H))))
            big = np.abs(h) > 1e-3 / H
            worst_rel = max(worst_rel, float(np.max(d[big] / np.abs(h[big]))))
        print(f"H={H:3d} h0_scale={h0:.0f}: worst {worst:.2e}  worst relative {worst_rel:.2e}  (gate 1e-5)")
