"""Development probe: per-phase cycles of g2k_encoder_chain_kernel from a
build with -DG2K_CHAIN_STAMPS (tools/ab/chain_stamps.so; the stamps land in
cost[s][f][33..41]).  python tools/probes/chain_stamps.py LIB.so"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from multimodaltraj_2_amd import _lib  # noqa: E402
from multimodaltraj_2_amd.encoder_step import EncoderChain  # noqa: E402
from test_encoder_chain_gpu import setup  # noqa: E402

_lib._lib = _lib.load(sys.argv[1])
gpu = torch.device("cuda:0")
names = ["h max", "cell", "B1", "E+exp,B2", "A/cost,B3", "As (w0)", "B4", "step", "store,B6"]
for H in (128, 512):
    S, F = 8, 20
    t, n_frames, G, params, cell, h0 = setup(gpu, S, F, H=H)
    n_frames = torch.full((S,), F, dtype=torch.int32, device=gpu)
    ch = EncoderChain(params, cell)
    for _ in range(3):
        out, _ = ch.run(t["pos"], t["vislet"], G, t["targets"], t["n_active"], n_frames, h0.clone(), stride=0)
    torch.cuda.synchronize()
    st = out.cost.reshape(S * F, 64)[:, 33:42].cpu().numpy()
    med = np.median(st[1:], axis=0)
    print(f"H {H}: cycles per frame (median) total {med.sum():.0f}: " +
          ", ".join(f"{n} {v:.0f}" for n, v in zip(names, med)))
