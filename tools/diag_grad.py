"""Diagnostic: the train-mode gradient (g2k_step_grad_f32) at one config.
1) time per launch (torch events, in-tree library) for each G2K_GRAD_GW;
2) phase timeline (s_memtime, shader cycles) of workgroup (0, 0) wave 0 from a
   separate -DG2K_STAMPS build in /tmp (never the shipped library)."""
import ctypes, os, subprocess, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import _lib, build, frame_step as fs, train_step as ts
from multimodaltraj_2_amd.synthetic import make_batch, CONFIGS

cfg = sys.argv[1] if len(sys.argv) > 1 else "eth_hotel_synth"
c = CONFIGS[cfg]
S = c["S"] if c["S"] <= 256 else c["S"] // 8
b = make_batch(S, c["Nmax"], c["H"])
dev = torch.device("cuda")
p = fs.init_params(c["Nmax"], device=dev)
t = b.to_device(dev)


def plan():
    return ts.GradPlan(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"])


ref = None
variants = [("seq", {}), ("wave GW4", {"G2K_GRAD_GW": "4"})]
for name, env in variants:
    for k in ("G2K_GRAD_GW", "G2K_GRAD_FPG"):
        os.environ.pop(k, None)
    os.environ.update(env)
    g = plan()
    for _ in range(5):
        g.run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        g.run()
    e1.record()
    torch.cuda.synchronize()
    out = g.grad.cpu().numpy()
    if ref is None:
        ref = out
    err = float(np.abs(out - ref).max() / np.abs(ref).max())
    print(f"{cfg} {name}: {e0.elapsed_time(e1) / 50 * 1e3:.1f} us per g2k_step_grad_f32 "
          f"(rel diff vs first {err:.1e})")
for k in ("G2K_GRAD_GW", "G2K_GRAD_FPG"):
    os.environ.pop(k, None)

out = "/tmp/libg2k_gstamps.so"
subprocess.run([build.HIPCC, *build.FLAGS, "-DG2K_STAMPS", "-o", out, *build.SRC], check=True)
lib = _lib.load(out)
_lib._lib = lib
lib.g2k_debug_stamps.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
g = plan()
for _ in range(3):
    g.run()
torch.cuda.synchronize()
st = (ctypes.c_ulonglong * 64)()
lib.g2k_debug_stamps(st, 64)
v = np.array(st[18:33], dtype=np.int64)
print("seq kernel WG(0,0): start->last frame top", int(v[1] - v[0]), "start->end", int(v[14] - v[0]))
idx = [19, 20, 21, 22, 24, 25, 26, 27, 28, 29, 30]
names = ["top", "B", "U/Ve", "E", "C", "M", "dY", "dM/dWo", "dC/dWc", "dE", "dU/sums"]
w = np.array([st[i] for i in idx], dtype=np.int64)
print("seq kernel WG(0,0), last frame, phase cycles:",
      ", ".join(f"{names[i]} {w[i] - w[i - 1]}" for i in range(1, len(w))),
      "| row + expansion", int(st[32] - st[30]))
