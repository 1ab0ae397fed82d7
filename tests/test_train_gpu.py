"""--mode train on the GPU: g2k_step_grad_f32 / g2k_update_f32 vs the float64
oracle (scene_loss_grad / optimizer_update, pinned by finite differences in
tests/test_train_oracle.py; unpinned against the reference, which has no
loss).  Tolerance (written here): per parameter block
max|g - ref| <= 1e-4 * max|ref| (normwise: fp32 sums over up to F x Nmax
terms); loss 1e-4 relative; count exact."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd import train_step as ts
from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch
from oracle import g2k_ref as ref
from tests.conftest import close

pytestmark = pytest.mark.gpu
TOL = 1e-4


def _ref_grad(b, w, nfr, mask, lam):
    R = {k: np.zeros(np.shape(w[k])) for k in ref.GRAD_ORDER}
    loss = cnt = 0
    for s in range(b.S):
        l, c, g = ref.scene_loss_grad(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s],
                                      b.n_active[s], n_frames=int(nfr[s]), lam=lam,
                                      ped_mask=None if mask is None else mask[s])
        loss += l
        cnt += c
        for k in R:
            R[k] += g[k]
    return loss, cnt, R


# Nmax 7 / 20 / 30: partial pedestrian tiles; Nmax 200 / 256: the dWo
# accumulation in frame order (one copy) instead of one copy per producer;
# F 40: two frame chunks
@pytest.mark.parametrize("Nmax,F,lam", [
    (32, 6, 5e-4), (7, 5, 0.05), (200, 3, 0.05), (32, 7, 0.05), (20, 9, 0.05), (64, 7, 5e-4),
    (256, 4, 0.05), (30, 40, 0.05)])
def test_grad_matches_oracle(gpu, Nmax, F, lam):
    S = 3
    b = make_batch(S, Nmax, 64, F=F, seed=21)
    mask = np.ones((S, Nmax), bool)
    mask[1, ::2] = False
    nfr = np.array([F, max(F - 2, 1), 0], np.int32)
    params = fs.init_params(Nmax, seed=0, device=gpu)
    t = b.to_device(gpu)
    gp = ts.GradPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                     n_frames=torch.from_numpy(nfr).to(gpu),
                     ped_mask=torch.from_numpy(mask.astype(np.uint8)).to(gpu), lam=lam)
    g = gp.run().cpu().numpy().astype(np.float64)
    loss, cnt, R = _ref_grad(b, params.numpy(), nfr, mask, lam)
    _check_grad(g, loss, cnt, R, Nmax)


def _check_grad(g, loss, cnt, R, Nmax):
    P = ts.grad_size(Nmax)
    assert g.shape == (P + 2,)
    off = 0
    for k in ref.GRAD_ORDER:
        r = R[k].reshape(-1)
        got = g[off:off + r.size]
        off += r.size
        if k == "Wr":
            assert np.all(got == 0)
        else:
            assert np.abs(got - r).max() <= TOL * np.abs(r).max(), k
    assert off == P
    assert abs(g[P] - loss) <= TOL * loss
    assert g[P + 1] == cnt


def test_grad_deterministic(gpu):
    b = make_batch(8, 32, 64, seed=5)
    params = fs.init_params(32, seed=0, device=gpu)
    t = b.to_device(gpu)
    gp = ts.GradPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"])
    g1 = gp.run().clone()
    g2 = gp.run().clone()
    torch.cuda.synchronize()
    assert torch.equal(g1, g2)


@pytest.mark.parametrize("rms,clip", [(False, 0.0), (True, 10.0), (True, 0.5), (False, 0.5)])
def test_update_matches_oracle(gpu, rms, clip):
    rng = np.random.default_rng(3)
    P = 1264
    p = rng.standard_normal(P).astype(np.float32)
    g = (5 * rng.standard_normal(P + 2)).astype(np.float32)
    g[P + 1] = 7.0
    ms0 = np.abs(rng.standard_normal(P)).astype(np.float32)
    flat = torch.from_numpy(p).to(gpu)
    ms = torch.from_numpy(ms0).to(gpu) if rms else None
    ts.optimizer_update(flat, torch.from_numpy(g).to(gpu), lr=5e-3, decay=0.95, grad_clip=clip,
                        ms=ms)
    torch.cuda.synchronize()
    rp, rm = ref.optimizer_update(p, ms0 if rms else None, g[:P], g[P + 1], 5e-3, 0.95, clip)
    assert np.abs(flat.cpu().numpy() - rp).max() <= 1e-6 * max(1.0, np.abs(rp).max())
    if rms:
        assert np.abs(ms.cpu().numpy() - rm).max() <= 1e-5 * np.abs(rm).max()


@pytest.mark.parametrize("Nmax,S,F,rms", [(32, 8, 20, True), (7, 3, 5, False), (256, 4, 6, True),
                                           (200, 2, 4, True)])
def test_fused_grad_update_matches_two_calls(gpu, Nmax, S, F, rms):
    """g2k_step_grad_update_f32 == g2k_step_grad_f32 + g2k_update_f32, bit for
    bit (same reduction order, same update), grad [P + 2] included."""
    b = make_batch(S, Nmax, 64, F=F, seed=9)
    params = fs.init_params(Nmax, seed=0, device=gpu)
    t = b.to_device(gpu)
    out = []
    for fused in (False, True):
        flat, views = ts.flat_params(params)
        ms = torch.full_like(flat, 0.25) if rms else None
        gp = ts.GradPlan(views, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                         lam=0.05)
        if fused:
            g = gp.run_update(flat, ms, lr=5e-3, decay=0.95, grad_clip=10.0)
        else:
            g = gp.run()
            ts.optimizer_update(flat, g, lr=5e-3, decay=0.95, grad_clip=10.0, ms=ms)
        torch.cuda.synchronize()
        out.append((g.clone(), flat.clone(), None if ms is None else ms.clone()))
    (g0, p0, m0), (g1, p1, m1) = out
    assert torch.equal(g0, g1) and torch.equal(p0, p1)
    assert m0 is None or torch.equal(m0, m1)


def test_train_step_reduces_loss(gpu):
    b = make_batch(16, 32, 128, seed=8)
    params = fs.init_params(32, seed=0, device=gpu)
    t = b.to_device(gpu)
    step = ts.TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                        t["h0"])
    losses = []
    for _ in range(6):
        g = step.run()
        torch.cuda.synchronize()
        losses.append(float(g[-2]) / float(g[-1]))
    assert np.all(np.isfinite(losses))
    assert losses[-1] < losses[0]
    # the step's forward outputs are the reference-mode step on the updated weights
    assert torch.isfinite(step.out.pred).all() and torch.isfinite(step.out.h).all()


def _train_batch(gpu, S, Nmax, H, F=20, seed=3):
    b = make_batch(S, Nmax, H, F=F, seed=seed, h0_scale=1.0)
    params = fs.init_params(Nmax, seed=0, device=gpu)
    return b, params, b.to_device(gpu)


def test_train_step_outputs_match_forward_step(gpu):
    """g2k_train_step_f32: its pred / h are the reference-mode step's bit for
    bit (same tiles, same recurrence); the metric sums the same within the
    tolerance (the train kernel's producers own whole frames, so the sums
    run in another order); its gradient is g2k_step_grad_f32's bit for bit."""
    b, params, t = _train_batch(gpu, 6, 32, 128)
    args = (params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    o1 = fs.step_fused(*args)
    tp = ts.TrainPlan(*args)
    g = tp.run().clone()
    g2 = ts.GradPlan(*args[:6]).run().clone()
    torch.cuda.synchronize()
    assert torch.equal(o1.pred, tp.out.pred)
    assert torch.equal(o1.h, tp.out.h)
    assert close(tp.out.metrics.cpu().numpy(), o1.metrics.cpu().numpy()) <= TOL
    assert torch.equal(g, g2)


@pytest.mark.parametrize("name,S", [("eth_hotel_synth", 256), ("eth_ucy_loo_kfold4", 128),
                                    ("relational_attn_h256", 256), ("dense_crowd", 128)])
def test_train_config_shape_matches_oracle(gpu, name, S):
    """The loss gradient at each BASELINE config's benchmark shape: the
    all-scene sum [P + 2] against the oracle's, and every 16th scene's own
    gradient row (the workspace rows the sum is formed from)."""
    c = CONFIGS[name]
    Nmax, H = c["Nmax"], c["H"]
    b, params, t = _train_batch(gpu, S, Nmax, H, seed=1)
    tp = ts.TrainPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    g = tp.run().cpu().numpy().astype(np.float64)
    torch.cuda.synchronize()
    P = ts.grad_size(Nmax)
    X = 1 if S >= 256 else min(4, 256 // S)         # workgroups per scene (one row each)
    rows = (tp._ws[:S * X * (P + 2) * 4].view(torch.float32).reshape(S, X, P + 2)
            .double().sum(1).cpu().numpy())
    w = params.numpy()
    R = {k: np.zeros(np.shape(w[k])) for k in ref.GRAD_ORDER}
    loss = cnt = 0
    for s in range(S):
        l, cn, gs = ref.scene_loss_grad(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s],
                                        b.n_active[s], n_frames=b.F)
        loss += l
        cnt += cn
        for k in R:
            R[k] += gs[k]
        if s % 16 == 0:
            r = np.concatenate([np.asarray(gs[k]).reshape(-1) for k in ref.GRAD_ORDER])
            assert np.abs(rows[s, :P] - r).max() <= TOL * np.abs(r).max(), s
            assert abs(rows[s, P] - l) <= TOL * l and rows[s, P + 1] == cn
    _check_grad(g, loss, cnt, R, Nmax)


def test_train_step_world2_branch_matches_one_rank(gpu, monkeypatch):
    """TrainStep's multi-rank branch (gradient, all-reduce, separate update)
    driven on one GPU: with the all-reduce of a one-rank group (identity) it
    must give the one-call update bit for bit; with the scenes split into two
    halves and their gradients summed (what the all-reduce of two ranks
    does) the update agrees within the tolerance."""
    b, params, t = _train_batch(gpu, 8, 32, 128)
    keys = ("pos", "vislet", "G", "targets", "n_active", "h0")
    one = ts.TrainStep(params, *(t[k] for k in keys))
    g1 = one.run().clone()
    p1 = one.flat.clone()
    two = ts.TrainStep(params, *(t[k] for k in keys))
    two.world = 2
    monkeypatch.setattr(ts, "allreduce_grad", lambda buf, group=None: buf)
    g2 = two.run().clone()
    torch.cuda.synchronize()
    assert torch.equal(g1, g2) and torch.equal(p1, two.flat)
    # two halves, gradients summed as the all-reduce would, one update
    flat, views = ts.flat_params(params)
    ms = torch.ones_like(flat)
    gs = []
    for lo, hi in ((0, 4), (4, 8)):
        h = {k: t[k][lo:hi].contiguous() for k in keys}
        gs.append(ts.TrainPlan(views, *(h[k] for k in keys)).run().clone())
    gsum = gs[0] + gs[1]
    ts.optimizer_update(flat, gsum, ms=ms)
    torch.cuda.synchronize()
    P = flat.numel()
    gn, gr = gsum.cpu().numpy(), g1.cpu().numpy()
    assert np.abs(gn[:P] - gr[:P]).max() <= 1e-5 * np.abs(gr[:P]).max()
    assert gn[P + 1] == gr[P + 1]
    assert np.abs(flat.cpu().numpy() - p1.cpu().numpy()).max() <= 1e-5


# The recurrence waves' gradient frames (the last R = 4 own frames of the
# last chunk once it holds 2 NP or more) split by tile with producers 0..R-1
# (g2k_scene.hip grad_rec_tiles), checked against the oracle: 3 tiles (an odd
# split, Nmax 48 with 33+ active), Nmax 256 (dWo^T added in frame order
# across recurrence waves and producers, dwo_seq), the NLL loss, and H = 512
# (the 4-producer train build, whose recurrence waves form As but not M of
# the first frames: the producers publish M only with the cost the gradient
# terms read).  Through the train step (h_in given: the recurrence runs).
@pytest.mark.parametrize("Nmax,F,H,loss", [(48, 20, 128, "l2"), (256, 16, 128, "l2"),
                                           (48, 20, 128, "nll"), (48, 12, 512, "l2"),
                                           (64, 9, 512, "l2")])
def test_train_rec_frames_tile_split_matches_oracle(gpu, Nmax, F, H, loss):
    S = 3
    n_active = [Nmax, max(Nmax - 5, 33), 17]
    b = make_batch(S, Nmax, H, F=F, seed=41, n_active=n_active, h0_scale=1.0)
    nfr = np.array([F, F - 1, F], np.int32)
    mask = np.ones((S, Nmax), bool)
    mask[0, 3::7] = False
    params = fs.init_params(Nmax, seed=0, device=gpu)
    if loss == "nll":
        params.Wo.mul_(0.05)
        params.head = torch.from_numpy((0.3 * np.random.default_rng(5).standard_normal((3, 12)))
                                       .astype(np.float32)).to(gpu)
    t = b.to_device(gpu)
    kw = dict(n_frames=torch.from_numpy(nfr).to(gpu),
              ped_mask=torch.from_numpy(mask.astype(np.uint8)).to(gpu), lam=0.05)
    tp = ts.TrainPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                      loss=loss, **kw)
    g = tp.run().cpu().numpy().astype(np.float64)
    w = params.numpy()
    order = ref.GRAD_ORDER + (("head",) if loss == "nll" else ())
    R = {k: 0.0 for k in order}
    lsum = cnt = 0
    for s in range(S):
        l_, c_, gg = ref.scene_loss_grad(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s],
                                         b.n_active[s], n_frames=int(nfr[s]), lam=0.05,
                                         ped_mask=mask[s], loss=loss, head=w.get("head"))
        lsum += l_
        cnt += c_
        for k in order:
            R[k] = R[k] + gg[k]
    off = 0
    for k in order:
        r = np.asarray(R[k]).reshape(-1)
        got = g[off:off + r.size]
        off += r.size
        if k == "Wr":
            assert np.all(got == 0)
        else:
            assert np.abs(got - r).max() <= TOL * np.abs(r).max(), k
    assert off == ts.grad_size(Nmax, loss)
    assert abs(g[off] - lsum) <= TOL * abs(lsum) and g[off + 1] == cnt
    # the forward outputs of the same launch: pred and h as the forward step's
    fwd = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                        **kw)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(tp.out.pred.cpu().numpy(), fwd.pred.cpu().numpy())
    np.testing.assert_array_equal(tp.out.h.cpu().numpy(), fwd.h.cpu().numpy())
