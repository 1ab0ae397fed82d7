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
from multimodaltraj_2_amd.synthetic import make_batch
from oracle import g2k_ref as ref

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


# G2K_GRAD_FPG forces frames per workgroup (the launcher picks 1 for these
# small S): groups of 2/3/8 frames exercise the prefetch double buffer, the
# frame-order row accumulation and n_frames ending inside a group;
# G2K_GRAD_GW selects the one-wave-per-frame kernel
@pytest.mark.parametrize("Nmax,F,lam,env", [
    (32, 6, 5e-4, {}), (7, 5, 0.05, {}), (200, 3, 0.05, {}),
    (32, 7, 0.05, {"G2K_GRAD_FPG": "3"}), (20, 9, 0.05, {"G2K_GRAD_FPG": "2"}),
    (64, 7, 5e-4, {"G2K_GRAD_FPG": "8"}), (256, 4, 0.05, {"G2K_GRAD_FPG": "3"}),
    (32, 6, 5e-4, {"G2K_GRAD_GW": "4"}), (200, 3, 0.05, {"G2K_GRAD_GW": "2"})])
def test_grad_matches_oracle(gpu, monkeypatch, Nmax, F, lam, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
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
