"""GPU: train mode with the bivariate-Gaussian NLL as the loss
(G2K_STEP_LOSS_NLL; north_star: "the bivariate-Gaussian NLL loss" fused into
the per-frame pipeline).  The scene kernel's producer tiles turn each
prediction tile's pairs into the NLL and d nll / d pred (the head's per-step
sigma_x, sigma_y, rho) and the head's own gradient, in the same launch as the
forward outputs.  Checked against the float64 oracle scene_loss_grad(loss=
"nll"), itself pinned by central finite differences
(tests/test_train_oracle.py); PARITY UNPINNED against the reference, which has
no loss.  Tolerance (written here): per parameter block max|g - ref| <= 1e-4 *
max|ref|; loss 1e-4 relative; count exact."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd import train_step as ts
from multimodaltraj_2_amd.synthetic import make_batch
from oracle import g2k_ref as ref

pytestmark = pytest.mark.gpu
TOL = 1e-4
ORDER = ref.GRAD_ORDER + ("head",)


def _params(Nmax, gpu, seed=0):
    p = fs.init_params(Nmax, seed=seed, device=gpu)
    p.Wo.mul_(0.05)                                   # predictions of O(1): a sane NLL
    p.head = torch.from_numpy((0.3 * np.random.default_rng(seed + 1).standard_normal((3, 12)))
                              .astype(np.float32)).to(gpu)
    return p


def _ref(b, w, nfr, mask, lam, stride=1, targets=None):
    R = {k: 0.0 for k in ORDER}
    loss = cnt = 0
    for s in range(b.S):
        l, c, g = ref.scene_loss_grad(b.pos[s], b.vislet[s], b.G[s], w,
                                      b.targets[s] if targets is None else targets[s],
                                      b.n_active[s], n_frames=int(nfr[s]), lam=lam, stride=stride,
                                      ped_mask=None if mask is None else mask[s], loss="nll",
                                      head=w["head"])
        loss += l
        cnt += c
        for k in ORDER:
            R[k] = R[k] + g[k]
    return loss, cnt, R


def _check(g, loss, cnt, R, Nmax):
    P = ts.grad_size(Nmax, "nll")
    assert g.shape == (P + 2,)
    off = 0
    for k in ORDER:
        r = np.asarray(R[k]).reshape(-1)
        got = g[off:off + r.size]
        off += r.size
        if k == "Wr":
            assert np.all(got == 0)
        else:
            assert np.abs(got - r).max() <= TOL * np.abs(r).max(), k
    assert off == P
    assert abs(g[P] - loss) <= TOL * abs(loss)
    assert g[P + 1] == cnt


@pytest.mark.parametrize("Nmax,F,H", [(32, 7, 64), (20, 9, 128), (64, 5, 256), (7, 4, 64)])
def test_nll_grad_matches_oracle(gpu, Nmax, F, H):
    S = 3
    b = make_batch(S, Nmax, H, F=F, seed=31)
    mask = np.ones((S, Nmax), bool)
    mask[1, ::3] = False
    nfr = np.array([F, max(F - 2, 1), 0], np.int32)
    params = _params(Nmax, gpu)
    t = b.to_device(gpu)
    kw = dict(n_frames=torch.from_numpy(nfr).to(gpu),
              ped_mask=torch.from_numpy(mask.astype(np.uint8)).to(gpu), lam=0.05)
    g = ts.GradPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                    loss="nll", **kw).run().cpu().numpy().astype(np.float64)
    _check(g, *_ref(b, params.numpy(), nfr, mask, 0.05), Nmax)
    # the same from the train step (forward outputs + gradient in one launch),
    # pedestrian-major pred: identical gradient, and forward outputs as L2 mode's
    tp = ts.TrainPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                      loss="nll", pred_layout="ped", **kw)
    g2 = tp.run().cpu().numpy().astype(np.float64)
    np.testing.assert_array_equal(g2, g)
    fwd = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                        n_frames=kw["n_frames"], ped_mask=kw["ped_mask"], lam=0.05)
    # (the metric sums' order differs: train mode's workers own whole frames)
    np.testing.assert_allclose(tp.out.metrics.cpu().numpy(), fwd.metrics.cpu().numpy(), rtol=1e-6)
    np.testing.assert_array_equal(tp.out.h.cpu().numpy(), fwd.h.cpu().numpy())


def test_nll_shared_targets_stride0(gpu):
    """Real-data form: stride-0 windows, one target set for every frame."""
    S, Nmax, F = 4, 32, 6
    b = make_batch(S, Nmax, 64, F=F, seed=33)
    t = b.to_device(gpu)
    pos = t["pos"][:, :8].contiguous()
    tg1 = t["targets"][:, :1].contiguous()
    params = _params(Nmax, gpu, seed=2)
    g = ts.GradPlan(params, pos, t["vislet"], t["G"], tg1, t["n_active"], stride=0, lam=0.05,
                    loss="nll", targets_shared=True, frames=F).run().cpu().numpy().astype(np.float64)
    rep = np.repeat(b.targets[:, :1], F, axis=1)
    b.pos = b.pos[:, :8]
    _check(g, *_ref(b, params.numpy(), [F] * S, None, 0.05, stride=0, targets=rep), Nmax)


def test_nll_train_step_reduces_loss(gpu):
    S, Nmax = 16, 32
    b = make_batch(S, Nmax, 64, F=10, seed=35)
    t = b.to_device(gpu)
    params = _params(Nmax, gpu, seed=3)
    step = ts.TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                        loss="nll", lr=0.01)
    assert step.P == ts.grad_size(Nmax, "nll")
    losses = []
    for _ in range(30):
        g = step.run()
        losses.append(float(g[-2] / g[-1]))
    assert all(b_ < a_ for a_, b_ in zip(losses, losses[1:])), losses[::5]   # descends every step
    assert losses[-1] < 0.95 * losses[0], losses[::5]
    # the head is trained too
    head = step.flat[ts.grad_size(Nmax):].cpu().numpy()
    assert np.abs(head - params.head.reshape(-1).cpu().numpy()).max() > 1e-3
