"""Diagnostic: timeline (shader cycles, low 32 bits of s_memtime) of scene-kernel
workgroups 0, 85, 170, 255 — prologue, staging barriers, per-frame producer
flags, per-frame recurrence completion, producer chunk ends.  Builds a
separate -DG2K_STAMPS_SCENE library into /tmp; never the shipped one.
Extra -D flags: G2K_DIAG_FLAGS (comma separated), e.g. -DG2K_DIAG_TWICE."""
import ctypes, os, subprocess, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import _lib, build, frame_step as fs
from multimodaltraj_2_amd.synthetic import make_batch, CONFIGS

extra = [f for f in os.environ.get("G2K_DIAG_FLAGS", "").split(",") if f]
out = "/tmp/libg2k_sstamps.so"
subprocess.run([build.HIPCC, *build.FLAGS, "-DG2K_STAMPS_SCENE", *extra, "-o", out, *build.SRC],
               check=True)
lib = _lib.load(out)
_lib._lib = lib
lib.g2k_debug_sstamps.argtypes = [ctypes.POINTER(ctypes.c_uint)]
cfg = sys.argv[1] if len(sys.argv) > 1 else "eth_hotel_synth"
c = CONFIGS[cfg]
S = c["S"] if c["S"] <= 256 else c["S"] // 8
b = make_batch(S, c["Nmax"], c["H"])
dev = torch.device("cuda")
p = fs.init_params(c["Nmax"], device=dev)
t = b.to_device(dev)
for _ in range(10):
    o = fs.step_fused(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
torch.cuda.synchronize()
st = (ctypes.c_uint * 512)()
lib.g2k_debug_sstamps(st)
raw = np.array(st[:], dtype=np.int64).reshape(4, 128)
F = b.F
for k in range(4):
    blk = 85 * k
    if blk >= S:
        continue
    r = np.where(raw[k] == 0xFFFFFFFF, -1, (raw[k] - raw[k, 0]) % (1 << 32))
    print(f"== WG {blk} n_active={b.n_active[blk]}: start {r[0]} dma-issued {r[103]} nf-known {r[104]} vmcnt {r[102]} B1 {r[1]} B2 {r[2]} end {r[100]}")
    print("   prologue: args-ready", r[92], "pos-dma-issued", r[93], "segs-issued", r[94], " epilogue: B3", r[95], "B4", r[96], "h-stored", r[97])
    print("   rec heads done w0..3:", " ".join(str(x) for x in r[74:78]))
    print("   staging tasks done:", " ".join(str(x) for x in r[105:109]), " rec init done:", r[113], " vtile0 entry/loop-end:", r[114], r[115])
    print("   producer flags:", " ".join(str(x) for x in r[3:3 + F]))
    print("   recur done    :", " ".join(str(x) for x in r[40:40 + F]))
    print("   recur per-frame:", " ".join(str(x) for x in np.diff(r[40:40 + F])))
    print("   wave chunk end:", " ".join(str(x) for x in r[80:80 + 12]))
    print("   frame10 poll-start w0..3:", " ".join(str(x) for x in r[116:120]))
    print("   frame10 poll-done  w0..3:", " ".join(str(x) for x in r[120:124]))
    print("   frame10 published  w0..3:", " ".join(str(x) for x in r[124:128]))
    rt = (raw[k, 99] - raw[k, 98]) % (1 << 32)
    print(f"   realtime start->end: {rt} ticks of 10 ns = {rt * 10} ns; shader-clock ticks {r[100]} -> {r[100] / max(rt * 10, 1):.3f} GHz")
    hw = raw[k, 60:72]
    print("   wave SIMD ids:", " ".join(str((int(h) >> 4) & 3) for h in hw), " CU", (int(hw[0]) >> 8) & 15, "SE", (int(hw[0]) >> 13) & 7)
    if raw[k, 73] != 0xFFFFFFFF:
        print(f"   repeat loop: {(int(raw[k, 73]) - int(raw[k, 72])) % (1 << 32) / 1000:.1f} cycles/frame")
