"""Diagnostic ablation of the recurrence kernel: builds variants with parts
removed (-DG2K_ABL=mask; results intentionally wrong) and times
g2k_frame_recurrence_f32 (S=256, F=20, H=128) for each, interleaved."""
import ctypes, os, subprocess, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import _lib, build

variants = {"base": 0, "no-permlane": 1, "no-barrier": 2, "no-zread": 4, "no-mfma": 8,
            "no-transpose": 16, "no-exp": 32, "none-of-above": 63}
libs = {}
for name, m in variants.items():
    out = f"/tmp/libg2k_abl{m}.so"
    subprocess.run([build.HIPCC, *build.FLAGS, f"-DG2K_ABL={m}", "-o", out, *build.SRC], check=True)
    libs[name] = _lib.load(out)
dev = torch.device("cuda")
S, F, H = 256, 20, int(os.environ.get("H", "128"))
A = torch.randn(S, F, 16, 16, device=dev)
h = torch.zeros(S, 16, H, device=dev)
res = {k: [] for k in variants}
for rnd in range(5):
    for name, lib in libs.items():
        d = _lib.G2KDims(S, F, 8, 12, 16, H, 1, 8, 0)
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(3):
            lib.g2k_frame_recurrence_f32(ctypes.byref(d), A.data_ptr(), h.data_ptr(), F, st)
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(50):
            lib.g2k_frame_recurrence_f32(ctypes.byref(d), A.data_ptr(), h.data_ptr(), F, st)
        e1.record(); torch.cuda.synchronize()
        res[name].append(e0.elapsed_time(e1) / 50 * 1e3)
for k, v in res.items():
    print(f"{k:14s} median {np.median(v):7.2f} us")
