"""Tuning: time g2k_step_fused_f32 with 4 vs 8 recurrence waves per scene
(G2K_RECUR_WAVES), interleaved rounds in one process (guide §5.4 rule 24)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch

dev = torch.device("cuda")
for cfg in sys.argv[1:] or ["eth_hotel_synth"]:
    c = CONFIGS[cfg]
    S = c["S"] if c["S"] <= 256 else c["S"] // 8
    b = make_batch(S, c["Nmax"], c["H"])
    p = fs.init_params(c["Nmax"], device=dev)
    t = b.to_device(dev)
    res = {}
    for rnd in range(5):
        for nw in ("4", "8"):
            os.environ["G2K_RECUR_WAVES"] = nw
            for _ in range(3):
                fs.step_fused(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
            e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
            e0.record()
            for _ in range(50):
                fs.step_fused(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
            e1.record(); torch.cuda.synchronize()
            res.setdefault(nw, []).append(e0.elapsed_time(e1) / 50 * 1e3)
    print(cfg, {k: f"median {np.median(v):.1f} us min {min(v):.1f}" for k, v in res.items()})
