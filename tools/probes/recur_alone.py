"""Per-frame cost of the recurrence alone (g2k_frame_recurrence_f32: the
barrier-exchange form, no producer waves): HIP-event time at F = 20 and F =
120 over S = 256 scenes, H = 128 -> cycles per frame (at the measured clock)."""
import sys
import torch
sys.path.insert(0, ".")
from multimodaltraj_2_amd import frame_step as fs  # noqa: E402


def t(F, S=256, H=128, reps=50):
    dev = torch.device("cuda")
    A = torch.randn(S, F, 16, 16, device=dev)
    h = torch.rand(S, 16, H, device=dev)
    for _ in range(5):
        fs.frame_recurrence(A, h)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fs.frame_recurrence(A, h)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


if __name__ == "__main__":
    if len(sys.argv) > 1:            # a variant library (tools/ab/libg2k_<name>.so)
        from multimodaltraj_2_amd import _lib
        _lib._lib = _lib.load(sys.argv[1])
        print("library", sys.argv[1])
    for H in (128, 256):
        a, b = t(20, H=H), t(120, H=H)
        print(f"recurrence alone H={H}: F=20 {a:.2f} us, F=120 {b:.2f} us -> {(b - a) / 100 * 1e3:.1f} ns/frame "
              f"(~{(b - a) / 100 * 2.1e3:.0f} cycles at 2.1 GHz)")
