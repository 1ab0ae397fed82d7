"""GPU: split scenes (G2K_STEP_SPLIT, include/g2k_hip.h).

A launch of fewer scenes than the device has CUs spreads each scene's frames
over X workgroups (workgroup x owns the frames g = x mod X; the first also
runs the recurrence).  Every per-frame output is computed by the same
arithmetic whatever X is, so pred, h, A and cost must be bit-identical to the
one-workgroup launch; the metric sums and the gradient are sums over frames
whose order changes with X (fixed for a given X: deterministic), so they are
held to the oracle's tolerances against X = 1 here and to the oracle itself
in test_step_gpu / test_train_gpu (whose small-S cases run split).  The
per-scene tickets in the workspace are zeroed on the stream by every launch
(ABI 7): a workspace poisoned with arbitrary bytes before any call — a
caller's uninitialised buffer, an aborted launch's leftovers — must give the
same results on the first and every later call."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd import train_step as ts
from multimodaltraj_2_amd.synthetic import make_batch

pytestmark = pytest.mark.gpu


def _n_frames(S, F, seed):
    """Frames per scene including 0 and fewer than X (a workgroup with no frame)."""
    nf = np.random.default_rng(seed).integers(0, F + 1, S).astype(np.int32)
    nf[:4] = [F, 0, 1, 3][:min(4, S)]
    return nf


@pytest.mark.parametrize("coresident", [False, True])
@pytest.mark.parametrize("S,Nmax,H,F", [(6, 32, 128, 20), (5, 64, 256, 20), (3, 30, 64, 41),
                                        (4, 256, 256, 9)])
def test_forward_split_equals_one_workgroup(gpu, S, Nmax, H, F, coresident):
    """coresident: the 8-wave geometry (G2K_STEP_CORESIDENT) split explicitly."""
    b = make_batch(S, Nmax, H, F=F, seed=11, h0_scale=1.0)
    t = b.to_device(gpu)
    params = fs.init_params(Nmax, seed=0, device=gpu)
    nfr = torch.from_numpy(_n_frames(S, F, 3)).to(gpu)
    outs = {}
    for X in (1, 2, 3, 4):
        plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                           t["h0"], n_frames=nfr, want_attn=True, pred_layout="ped", split=X,
                           coresident=coresident)
        runs = []
        ws = plan._keep[-1]
        for i in range(3):                     # every launch zeroes its tickets itself
            ws.random_(0, 256)                 # poisoned tickets and partials
            o = plan.run()
            torch.cuda.synchronize()
            runs.append({k: getattr(o, k).cpu().numpy().copy() for k in
                         ("pred", "h", "metrics", "attn", "cost")})
        for r in runs[1:]:
            for k in r:
                np.testing.assert_array_equal(r[k], runs[0][k])    # deterministic per X
        outs[X] = runs[0]
    nf = nfr.cpu().numpy()
    for X in (2, 3, 4):
        for s in range(S):
            n, f = int(b.n_active[s]), int(nf[s])
            for k in ("pred", "attn", "cost"):
                np.testing.assert_array_equal(outs[X][k][s, :f], outs[1][k][s, :f])
            assert np.array_equal(outs[X]["pred"][s, :f, :n], outs[1]["pred"][s, :f, :n])
        np.testing.assert_array_equal(outs[X]["h"], outs[1]["h"])
        m1, mx = outs[1]["metrics"], outs[X]["metrics"]
        assert np.all(np.abs(mx - m1) <= 1e-5 * np.maximum(1.0, np.abs(m1))), X
        np.testing.assert_array_equal(mx[:, 5], nf.astype(np.float32))   # frames


@pytest.mark.parametrize("S,Nmax,F,loss", [(6, 32, 20, "l2"), (3, 32, 40, "l2"), (4, 256, 9, "l2"),
                                           (5, 64, 36, "nll")])
def test_train_split_matches_one_workgroup(gpu, S, Nmax, F, loss):
    """F = 40 / 36: the own frames of a workgroup reach 2 NP, so its recurrence
    waves take gradient frames; Nmax 256: dWo^T added in own-frame order
    (dwo_seq); n_frames from 0 up."""
    b = make_batch(S, Nmax, 128, F=F, seed=13)
    t = b.to_device(gpu)
    nfr = torch.from_numpy(_n_frames(S, F, 5)).to(gpu)
    res = {}
    for X in (1, 2, 4):
        params = fs.init_params(Nmax, seed=0, device=gpu)
        if loss == "nll":
            params.head = torch.from_numpy(
                np.random.default_rng(1).normal(0.0, 0.3, (3, 12)).astype(np.float32)).to(gpu)
        tp = ts.TrainPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                          n_frames=nfr, lam=0.05, loss=loss, split=X)
        g = []
        for _ in range(2):
            tp._ws.random_(0, 256)            # poisoned rows, tickets and partials
            g.append(tp.run().clone())
        torch.cuda.synchronize()
        assert torch.equal(g[0], g[1])                                  # deterministic per X
        res[X] = (g[0].double().cpu().numpy(), tp.out.h.cpu().numpy().copy(),
                  tp.out.pred.cpu().numpy().copy())
    g1, h1, p1 = res[1]
    for X in (2, 4):
        gx, hx, px = res[X]
        # normwise per the oracle tests' bound; loss and count exact to 1e-5
        assert np.abs(gx[:-2] - g1[:-2]).max() <= 1e-5 * np.abs(g1[:-2]).max(), X
        assert abs(gx[-2] - g1[-2]) <= 1e-5 * abs(g1[-2]) and gx[-1] == g1[-1]
        np.testing.assert_array_equal(hx, h1)
        np.testing.assert_array_equal(px, p1)


def test_automatic_split_runs_the_recurrence_once(gpu):
    """S = 1 (automatic X = 4): h from the one recurrence, equal to X = 1."""
    b = make_batch(1, 32, 128, F=20, seed=2, h0_scale=1.0)
    t = b.to_device(gpu)
    params = fs.init_params(32, seed=0, device=gpu)
    a = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    o = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                      split=1)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a.h.cpu().numpy(), o.h.cpu().numpy())
    np.testing.assert_array_equal(a.pred.cpu().numpy(), o.pred.cpu().numpy())


def test_split_plan_on_a_side_stream_right_after_building(gpu):
    """The workspace's first zero-fill is ordered on the plan's own stream
    (frame_step.workspace), so a split plan launched on a side stream right
    after it is built — no synchronize in between, as bench.py's warm-up does
    over two streams — sees zeroed tickets: its metrics equal the same plan's
    on the current stream, and the tickets end at zero."""
    S, Nmax, H, F = 8, 32, 128, 20
    b = make_batch(S, Nmax, H, F=F, seed=21)
    t = b.to_device(gpu)
    params = fs.init_params(Nmax, seed=0, device=gpu)
    want = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                         t["h0"], split=4)
    torch.cuda.synchronize()
    # fill the caching allocator with non-zero blocks the workspace may reuse
    junk = [torch.full((1 << 16,), 255, dtype=torch.uint8, device=gpu) for _ in range(8)]
    del junk
    side = torch.cuda.Stream(device=gpu)
    plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                       split=4, stream=side)
    for _ in range(3):
        plan.run()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(plan.out.metrics.cpu().numpy(), want.metrics.cpu().numpy())
    assert fs.step_split(S, F, H, Nmax, t["pos"].shape[1], b.stride) == min(4, 256 // S)


def test_workspace_init_zero_fills_on_the_stream(gpu):
    """g2k_workspace_init: the C caller's stream-ordered first fill."""
    import ctypes
    from multimodaltraj_2_amd import _lib
    ws = torch.full((4096,), 7, dtype=torch.uint8, device=gpu)
    s = torch.cuda.Stream(device=gpu)
    s.wait_stream(torch.cuda.current_stream())
    rc = _lib.load().g2k_workspace_init(ws.data_ptr(), 4096, ctypes.c_void_p(s.cuda_stream))
    assert rc == 0
    s.synchronize()
    assert int(ws.count_nonzero()) == 0
