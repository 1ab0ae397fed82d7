"""Per-frame cost of the standalone recurrence (g2k_frame_recurrence_f32,
S = 256 scenes): times F = 10, 20, 40 frames and reports the slope (us per
frame), for 4 and 8 recurrence waves (G2K_RECUR_WAVES), interleaved rounds."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import _lib

lib = _lib.load()
dev = torch.device("cuda")
S = 256
for H in (int(x) for x in (sys.argv[1:] or ["128"])):
    res = {}
    for rnd in range(5):
        for nw in ("4", "8"):
            os.environ["G2K_RECUR_WAVES"] = nw
            for F in (10, 20, 40):
                A = torch.randn(S, F, 16, 16, device=dev)
                h = torch.rand(S, 16, H, device=dev)
                d = _lib.G2KDims(S, F, 8, 12, 16, H, 1, 8, 0)
                st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
                for _ in range(3):
                    lib.g2k_frame_recurrence_f32(ctypes.byref(d), A.data_ptr(), h.data_ptr(), F, st)
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                for _ in range(50):
                    lib.g2k_frame_recurrence_f32(ctypes.byref(d), A.data_ptr(), h.data_ptr(), F, st)
                e1.record(); torch.cuda.synchronize()
                res.setdefault((nw, F), []).append(e0.elapsed_time(e1) / 50 * 1e3)
    for nw in ("4", "8"):
        m = {F: np.median(res[(nw, F)]) for F in (10, 20, 40)}
        slope = (m[40] - m[10]) / 30
        print(f"H={H} waves={nw}: F=10 {m[10]:.2f} us, F=20 {m[20]:.2f} us, F=40 {m[40]:.2f} us; "
              f"{slope * 1e3:.0f} ns/frame")
