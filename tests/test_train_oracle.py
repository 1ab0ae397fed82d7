"""The train-mode restatement (oracle/g2k_ref.py scene_loss_grad,
optimizer_update) pinned by central finite differences of its own float64
forward — the reference defines no loss (SURVEY.md finding 5), so nothing
else can pin it.  pred is linear in each single parameter (Wi, Wii, Wv, bv,
Wc, Wo), so the loss is quadratic in each and central differences are exact
up to rounding."""
import numpy as np
import pytest

from multimodaltraj_2_amd.synthetic import make_batch
from oracle import g2k_ref as ref


def _weights(nmax, seed=0):
    rng = np.random.default_rng(seed)
    shapes = dict(Wi=(nmax, 16), Wii=(16, 8), Wv=(8, 18), bv=(16,), Wr=(8, 2), Wc=(24, 8),
                  Wo=(8, nmax))
    return {k: rng.standard_normal(s) for k, s in shapes.items()}


@pytest.mark.parametrize("lam", [5e-4, 0.05])
def test_grad_matches_finite_differences(lam):
    Nmax, n = 8, 6
    b = make_batch(1, Nmax, 64, F=3, seed=3, n_active=[n])
    w = _weights(Nmax)
    mask = np.ones(Nmax, bool)
    mask[2] = False
    args = (b.pos[0], b.vislet[0], b.G[0])
    kw = dict(n_frames=3, lam=lam, ped_mask=mask)
    loss, cnt, g = ref.scene_loss_grad(*args, w, b.targets[0], n, **kw)
    assert cnt == 3 * (n - 1)
    rng = np.random.default_rng(1)
    for k in ref.GRAD_ORDER:
        for _ in range(4):
            idx = tuple(int(rng.integers(0, s)) for s in w[k].shape)
            h = 1e-3 * max(1.0, abs(w[k][idx]))
            wp = {kk: v.copy() for kk, v in w.items()}
            wm = {kk: v.copy() for kk, v in w.items()}
            wp[k][idx] += h
            wm[k][idx] -= h
            fd = (ref.scene_loss(*args, wp, b.targets[0], n, **kw)
                  - ref.scene_loss(*args, wm, b.targets[0], n, **kw)) / (2 * h)
            assert abs(fd - g[k][idx]) <= 1e-7 * max(1.0, abs(loss)), (k, idx, fd, g[k][idx])
    assert np.all(g["Wr"] == 0)
    assert np.all(g["Wi"][n:] == 0) and np.all(g["Wo"][:, n:] == 0)


def test_optimizer_update_clip_and_rmsprop():
    rng = np.random.default_rng(2)
    p = rng.standard_normal(50)
    g = 100 * rng.standard_normal(50)
    p1, _ = ref.optimizer_update(p, None, g, 4, 0.1, 0.95, 10.0)
    assert np.isclose(np.linalg.norm((p - p1) / 0.1), 10.0)        # clipped to the global norm
    p2, m = ref.optimizer_update(p, np.zeros(50), g, 4, 0.1, 0.95, 0.0)
    gg = g / 4
    assert np.allclose(m, 0.05 * gg * gg)
    assert np.allclose(p2, p - 0.1 * gg / np.sqrt(m + 1e-10))


def test_nll_loss_grad_matches_finite_differences():
    """loss = "nll": the bivariate-Gaussian NLL of the predictions (the
    build's; parity unpinned against the reference, which has no loss),
    pinned by central differences in every model parameter and the head.
    The NLL is not quadratic in the head, so the head uses a smaller step."""
    Nmax, n = 8, 6
    b = make_batch(1, Nmax, 64, F=2, seed=4, n_active=[n])
    w = _weights(Nmax, seed=5)
    for k in ("Wo", "Wc"):                    # pred of O(1): a well-conditioned NLL
        w[k] = 0.05 * w[k]
    head = 0.3 * np.random.default_rng(6).standard_normal((3, 12))
    mask = np.ones(Nmax, bool)
    mask[3] = False
    args = (b.pos[0], b.vislet[0], b.G[0])
    kw = dict(n_frames=2, lam=0.05, ped_mask=mask, loss="nll")
    loss, cnt, g = ref.scene_loss_grad(*args, w, b.targets[0], n, head=head, **kw)
    assert cnt == 2 * (n - 1)
    # the per-frame NLL equals bivariate_nll's (sample.py-side head) on the same pred
    fw = ref.frame_forward(b.pos[0][:8], b.vislet[0], b.G[0], w, 0.05, n)
    one, pairs, dh, _ = ref.bivariate_nll(fw["Y"][None], b.targets[0][:1], head, n, 1, mask)
    l1, _, g1 = ref.scene_loss_grad(*args, w, b.targets[0], n, head=head, **dict(kw, n_frames=1))
    assert np.isclose(one, l1, rtol=1e-12) and np.allclose(dh, g1["head"], rtol=1e-12)
    rng = np.random.default_rng(7)
    for k in ref.GRAD_ORDER + ("head",):
        for _ in range(4):
            base = head if k == "head" else w[k]
            idx = tuple(int(rng.integers(0, s)) for s in base.shape)
            h = (1e-5 if k == "head" else 1e-4) * max(1.0, abs(base[idx]))

            def f(delta):
                hh, ww = head.copy(), {kk: v.copy() for kk, v in w.items()}
                (hh if k == "head" else ww[k])[idx] += delta
                return ref.scene_loss(*args, ww, b.targets[0], n, head=hh, **kw)
            fd = (f(h) - f(-h)) / (2 * h)
            assert abs(fd - g[k][idx]) <= 1e-6 * max(1.0, abs(g[k][idx])), (k, idx, fd, g[k][idx])
    assert np.all(g["Wr"] == 0)
