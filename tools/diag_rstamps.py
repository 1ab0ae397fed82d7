"""Diagnostic: in-frame stamps of the recurrence (separate -DG2K_STAMPS_RECUR build)."""
import ctypes, os, subprocess, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import _lib, build, frame_step as fs
from multimodaltraj_2_amd.synthetic import make_batch

out = "/tmp/libg2k_rstamps.so"
subprocess.run([build.HIPCC, *build.FLAGS, "-DG2K_STAMPS_RECUR", "-o", out, *build.SRC], check=True)
lib = _lib.load(out)
_lib._lib = lib
for nw in sys.argv[1:] or ["4"]:
    os.environ["G2K_RECUR_WAVES"] = nw
    b = make_batch(256, 32, 128)
    dev = torch.device("cuda")
    p = fs.init_params(32, device=dev)
    t = b.to_device(dev)
    st = (ctypes.c_ulonglong * 16)()
    for _ in range(3):
        lib.g2k_debug_rstamps(st)
        fs.step_fused(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
        torch.cuda.synchronize()
    lib.g2k_debug_rstamps_get(st)
    v = np.array(st[:8], dtype=np.int64)
    names = ["z reads+B", "MFMA", "exp+P", "permlane sum", "publish", "stage(transpose)", "barrier"]
    print(f"waves={nw} frame total {v[7]-v[0]}:", {names[k]: int(v[k+1]-v[k]) for k in range(7)})
