"""Development probe (not product code): would a decoupled step — the
producers' kernel writing A to HBM, then a separate recurrence kernel on the
same stream — beat the fused kernel in the steady state?  The library
argument: a build whose g2k_step_fused_f32 drops h_in after binding (a
temporary one-line edit of g2k_abi.hip, `a.h_in = nullptr`: the scene
kernel's recurrence waves idle).  Result: profiles/r11g_decoupled_probe.txt.  eth_hotel_synth, 4 streams, co-resident,
graph-replayed, 200 steps.
    python tools/probes/decoupled_probe.py tools/ab/nochain.so"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from multimodaltraj_2_amd import _lib  # noqa: E402
from multimodaltraj_2_amd import frame_step as fs  # noqa: E402
from multimodaltraj_2_amd.synthetic import make_batch  # noqa: E402

dev = torch.device("cuda:0")
S, Nmax, H, F = 256, 32, 128, 20
b = make_batch(S, Nmax, H, F=F, seed=1)
NS, K = 4, 16


def build(want_attn):
    params = fs.init_params(Nmax, seed=0, device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(NS)]
    base = b.to_device(dev)
    plans, hs = [], []
    for k in range(K):
        t = {key: (v.clone() if isinstance(v, torch.Tensor) else v) for key, v in base.items()}
        p = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                        n_frames=t["n_frames"], ped_mask=t["ped_mask"], stride=b.stride,
                        stream=streams[k % NS], coresident=True, pred_layout="ped",
                        want_attn=want_attn)
        plans.append((p, t, streams[k % NS]))
        hs.append(t["h0"].clone())
    return plans, hs, streams


def timeit(step, streams, n=200, warm=20):
    el, _ = bench.timed_graph(step, n, warm, None, torch.cuda.synchronize, streams[0], side=streams[1:])
    return el / n * 1e6


res = {}
plans, hs, streams = build(False)
res["fused (tree lib)"] = timeit(lambda i: plans[i % K][0].run(), streams)
del plans
_lib._lib = _lib.load(sys.argv[1])
plans, hs, streams = build(True)
res["producers only (A out)"] = timeit(lambda i: plans[i % K][0].run(), streams)


def rec_only(i):
    p, t, st = plans[i % K]
    fs.frame_recurrence(p.out.attn, hs[i % K], stream=st)


res["recurrence kernel only"] = timeit(rec_only, streams)


def both(i):
    p, t, st = plans[i % K]
    p.run()
    fs.frame_recurrence(p.out.attn, hs[i % K], stream=st)


res["decoupled (producers, then g2k_recur_kernel)"] = timeit(both, streams)
for k, v in res.items():
    print(f"{k}: {v:.2f} us per step")
