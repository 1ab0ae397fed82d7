"""Diagnostic: per-stage s_memtime stamps of workgroup 0 of the fused step
(builds a separate -DG2K_STAMPS library into /tmp; never the shipped one)."""
import ctypes, os, subprocess, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import _lib, build, frame_step as fs
from multimodaltraj_2_amd.synthetic import make_batch, CONFIGS

out = "/tmp/libg2k_stamps.so"
subprocess.run([build.HIPCC, *build.FLAGS, "-DG2K_STAMPS", "-o", out, *build.SRC], check=True)
lib = _lib.load(out)
_lib._lib = lib
lib.g2k_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
names = {1: "A staging (weights, norms)", 2: "A V = norms @ Wi", 6: "A per-wave frames + reduce",
         11: "B metrics,h load,init,As DMA", 12: "B recurrence frames"}
for cfg in sys.argv[1:] or ["eth_hotel_synth"]:
    c = CONFIGS[cfg]
    S = c["S"] if c["S"] <= 256 else c["S"] // 8
    b = make_batch(S, c["Nmax"], c["H"])
    dev = torch.device("cuda")
    p = fs.init_params(c["Nmax"], device=dev)
    t = b.to_device(dev)
    for _ in range(5):
        o = fs.step_fused(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    torch.cuda.synchronize()
    st = (ctypes.c_ulonglong * 64)()
    lib.g2k_debug_stamps(st, 64)
    v = np.array(st[:13], dtype=np.int64)
    print(f"== {cfg} (S={S}) n_active[0]={b.n_active[0]}  frames-kernel WG(0,0) {v[6]-v[0]} ticks, "
          f"recur WG 0 {v[12]-v[10]} ticks")
    for k, k0 in ((1, 0), (2, 1), (6, 2), (11, 10), (12, 11)):
        print(f"  {names[k]:32s} {v[k]-v[k0]:8d}")
