"""The bivariate-Gaussian NLL head (csrc/g2k_nll.hip).
PARITY UNPINNED: the reference has no such head.  The oracle's gradient is
pinned by central finite differences (CPU); the HIP kernels are checked
against the oracle (GPU): nll / pair count / head gradient / d pred within
1e-4 relative, the sampler against the oracle's restatement of its hash and
Box-Muller draw."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd.synthetic import make_batch
from oracle import g2k_ref as ref
from tests.conftest import close

TOL = 1e-4


def _case(seed=0, F=3, N=6):
    rng = np.random.default_rng(seed)
    pred = rng.standard_normal((F, 24, N))
    tg = pred.reshape(F, 2, 12, N).transpose(0, 3, 2, 1) + 0.7 * rng.standard_normal((F, N, 12, 2))
    head = np.stack([0.3 * rng.standard_normal(12), 0.3 * rng.standard_normal(12),
                     0.8 * rng.standard_normal(12)])
    mask = np.ones(N, bool)
    mask[2] = False
    return pred, tg, head, mask


def test_oracle_gradient_finite_differences():
    pred, tg, head, mask = _case()
    nll, pairs, dh, dp = ref.bivariate_nll(pred, tg, head, 5, 2, mask)
    assert pairs == 2 * 4
    eps = 1e-6
    for idx in [(0, 0), (0, 11), (1, 5), (2, 3), (2, 9)]:
        hp, hm = head.copy(), head.copy()
        hp[idx] += eps
        hm[idx] -= eps
        fd = (ref.bivariate_nll(pred, tg, hp, 5, 2, mask)[0] - ref.bivariate_nll(pred, tg, hm, 5, 2, mask)[0]) / (2 * eps)
        assert abs(fd - dh[idx]) <= 1e-6 * max(1.0, abs(fd)), idx
    for idx in [(0, 0, 0), (1, 13, 4), (0, 11, 1), (1, 23, 3), (2, 5, 0)]:
        pp, pm = pred.copy(), pred.copy()
        pp[idx] += eps
        pm[idx] -= eps
        fd = (ref.bivariate_nll(pp, tg, head, 5, 2, mask)[0] - ref.bivariate_nll(pm, tg, head, 5, 2, mask)[0]) / (2 * eps)
        assert abs(fd - dp[idx]) <= 1e-6 * max(1.0, abs(fd)), idx


def test_oracle_sampler_moments():
    S, F, N = 2, 4, 256
    pred = np.zeros((S, F, 24, N))
    head = np.stack([np.full(12, np.log(2.0)), np.full(12, np.log(0.5)), np.full(12, np.arctanh(0.6))])
    x = ref.gauss_sample(pred, head, seed=12345)
    a, b = x[:, :, :12].ravel(), x[:, :, 12:].ravel()
    assert abs(a.mean()) < 0.05 and abs(b.mean()) < 0.0125
    assert abs(a.std() - 2.0) < 0.05 and abs(b.std() - 0.5) < 0.0125
    assert abs(np.corrcoef(a, b)[0, 1] - 0.6) < 0.02


@pytest.mark.gpu
def test_nll_kernel_matches_oracle(gpu):
    from multimodaltraj_2_amd.nll import GaussianHead
    b = make_batch(12, 32, 64, F=5, seed=9)
    S, F, N = 12, 5, 32
    rng = np.random.default_rng(4)
    pred = (np.transpose(b.targets, (0, 1, 4, 3, 2)).reshape(S, F, 24, N)
            + 0.05 * rng.standard_normal((S, F, 24, N))).astype(np.float32)
    pm = (rng.random((S, N)) > 0.2).astype(np.uint8)
    nf = rng.integers(0, F + 1, size=S).astype(np.int32)
    head = np.stack([np.log(0.05) + 0.2 * rng.standard_normal(12), np.log(0.05) + 0.2 * rng.standard_normal(12),
                     0.5 * rng.standard_normal(12)]).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)   # noqa: E731
    gh = GaussianHead(device=gpu)
    gh.head = t(head)
    nll, pairs, dh, dp = gh.nll(t(pred), t(b.targets), t(b.n_active), n_frames=t(nf), ped_mask=t(pm),
                                want_dpred=True)
    nll2, _, dh2, dp2 = gh.nll(t(pred), t(b.targets), t(b.n_active), n_frames=t(nf), ped_mask=t(pm),
                               want_dpred=True)
    torch.cuda.synchronize()
    assert torch.equal(dh, dh2) and torch.equal(nll, nll2) and torch.equal(dp, dp2)   # fixed order
    R_nll, R_pairs, R_dh, R_dp = 0.0, 0, np.zeros((3, 12)), np.zeros((S, F, 24, N))
    for s in range(S):
        l_, p_, h_, d_ = ref.bivariate_nll(pred[s], b.targets[s], head, int(b.n_active[s]), int(nf[s]),
                                           pm[s].astype(bool))
        R_nll += l_
        R_pairs += p_
        R_dh += h_
        R_dp[s] = d_
    assert int(pairs) == R_pairs
    assert abs(float(nll) - R_nll) <= TOL * abs(R_nll)
    assert np.abs(dh.cpu().numpy() - R_dh).max() <= TOL * np.abs(R_dh).max()
    assert close(dp.cpu().numpy(), R_dp) <= TOL


@pytest.mark.gpu
def test_gauss_sampler_matches_oracle(gpu):
    from multimodaltraj_2_amd.nll import GaussianHead
    rng = np.random.default_rng(2)
    pred = rng.standard_normal((3, 4, 24, 20)).astype(np.float32)
    head = np.stack([0.3 * rng.standard_normal(12), 0.3 * rng.standard_normal(12),
                     rng.standard_normal(12)]).astype(np.float32)
    gh = GaussianHead(device=gpu)
    gh.head = torch.from_numpy(head).to(gpu)
    seed = (7 << 32) + 99
    x = gh.sample(torch.from_numpy(pred).to(gpu), seed=seed).cpu().numpy()
    assert close(x, ref.gauss_sample(pred, head, seed)) <= TOL
    y = gh.sample(torch.from_numpy(pred).to(gpu), seed=seed + 1).cpu().numpy()
    assert not np.allclose(x, y)
