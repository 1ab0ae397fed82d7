"""Per-frame cost of the fused step's recurrence chain, without stamps: the
HIP-event time of g2k_step_fused_f32 at F = 8, 20, 32 frames (one LDS chunk) (S = 256, H = 128,
the producers' work per frame fixed by Nmax) -> the slope in ns and cycles per
frame.  Optional argv[1]: a variant library (tools/ab/libg2k_<name>.so)."""
import sys
import torch
sys.path.insert(0, ".")
from multimodaltraj_2_amd import _lib, frame_step as fs  # noqa: E402
from multimodaltraj_2_amd.synthetic import make_batch  # noqa: E402


def t_step(S, Nmax, H, F, reps=100, rot=4):
    dev = torch.device("cuda")
    params = fs.init_params(Nmax, seed=0, device=dev)
    plans = []
    for k in range(rot):
        b = make_batch(S, Nmax, H, F=F, seed=10 + k).to_device(dev)
        plans.append(fs.StepPlan(params, b["pos"], b["vislet"], b["G"], b["targets"], b["n_active"], b["h0"],
                                 n_frames=b["n_frames"], ped_mask=b["ped_mask"], pred_layout="ped"))
    for p in plans:
        p.run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for i in range(reps):
        plans[i % rot].run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


if __name__ == "__main__":
    if len(sys.argv) > 1:
        _lib._lib = _lib.load(sys.argv[1])
        print("library", sys.argv[1])
    for Nmax, H in ((32, 128), (4, 128), (64, 256)):
        ts = {F: t_step(256, Nmax, H, F) for F in (8, 20, 32)}
        slope = (ts[32] - ts[8]) / 24
        print(f"Nmax {Nmax} H {H}: " + "  ".join(f"F={F} {v:.2f} us" for F, v in ts.items()) +
              f"  -> {slope * 1e3:.0f} ns/frame (~{slope * 2.1e3:.0f} cycles at 2.1 GHz); "
              f"intercept {ts[20] - 20 * slope:.2f} us", flush=True)
