"""GPU a9 against the reference's OWN error code (tests/golden/errors_*.npz,
tools/make_error_fixtures.py: get_mean_error sample.py:21-82 and the
validation block train.py:636-674 run on real walk batches).

* g2k_ade_fde_f32 variant 0 on the fixture's predictions and targets, and the
  fused step g2k_step_fused_f32 on the fixture's INPUTS (window, vislet, G,
  weights: it forms its own predictions), reduced per batch
  (frame_step.batch_errors), against the reference's ADE_b and FDE_b for both
  divisors (leaveDataset 5 and the others);
* g2k_ade_fde_f32 variant 1 against get_mean_error's (ADE, FDE, counter).
Tolerance |got - ref| <= 1e-4 * max(1, |ref|).  Full-length targets only: the
GPU entry points take 12-point targets, the only lists the reference's loader
produces (quirk Q11); the short-target branch is pinned on the oracle
(tests/test_errors_golden.py)."""
import glob
import os

import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from tests.conftest import close

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "errors_*.npz")))
TOL = 1e-4


def val_inputs(z):
    """Per case: n, nb, pred band [24, n], paired targets [Nmax, 12, 2] (row
    i <-> the dict's i-th key, train.py:640) and the pairing mask."""
    out = []
    nmax = int(z["w_Wi"].shape[0])
    for c in range(int(z["val_count"])):
        p = f"val{c}_"
        n, nb = int(z[p + "n"]), int(z[p + "nb"])
        k = min(n, int(z[p + "K"]))
        tgt = np.zeros((nmax, 12, 2), np.float32)
        tgt[:k] = z[p + "heads"][:k]
        assert np.all(z[p + "lens"][:k] >= 12)
        mask = np.zeros(nmax, np.uint8)
        mask[:k] = 1
        out.append((p, n, nb, z[p + "pred"].reshape(24, n), tgt, mask))
    return out


def expected(z, p, n):
    return [(float(z[p + "ade_b"]), float(z[p + "fde_b"]), 2),
            (float(z[p + "ade_b5"]), float(z[p + "fde_b5"]), 5)]


def check_batches(z, cs, metrics):
    for s, (p, n, nb, _, _, mask) in enumerate(cs):
        for ade_r, fde_r, l in expected(z, p, n):
            ade, fde = fs.batch_errors(metrics[s:s + 1], leave_dataset=l, num_nodes=[n])
            if np.isnan(ade_r):
                assert mask.sum() == 0 and np.isnan(ade[0])
                continue
            assert close(ade[0], ade_r) <= TOL, (p, l, ade[0], ade_r)
            assert close(fde[0], fde_r) <= TOL, (p, l, fde[0], fde_r)


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p))
def test_ade_fde_variant0_vs_reference_code(gpu, path):
    z = np.load(path)
    cs = val_inputs(z)
    nmax = int(z["w_Wi"].shape[0])
    S, F = len(cs), max(c[2] for c in cs)
    pred = np.zeros((S, F, 24, nmax), np.float32)
    tgt = np.zeros((S, F, nmax, 12, 2), np.float32)
    mask = np.zeros((S, nmax), np.uint8)
    for s, (p, n, nb, band, t, m) in enumerate(cs):
        pred[s, :nb, :, :n] = band
        tgt[s] = t
        mask[s] = m
    na = torch.tensor([c[1] for c in cs], dtype=torch.int32, device=gpu)
    nf = torch.tensor([c[2] for c in cs], dtype=torch.int32, device=gpu)
    out = fs.ade_fde(torch.from_numpy(pred).to(gpu), torch.from_numpy(tgt).to(gpu), na,
                     n_frames=nf, ped_mask=torch.from_numpy(mask).to(gpu), variant=0)
    torch.cuda.synchronize()
    check_batches(z, cs, out)


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p))
@pytest.mark.parametrize("pred_layout", ["band", "ped"])
def test_fused_step_metrics_vs_reference_code(gpu, path, pred_layout):
    """The fused step on the fixture's inputs (node-slice / time-slice windows,
    one window per batch: stride 0, every frame of the batch re-fed the same
    inputs as train.py's validation loop does) forms its own predictions; its
    metric terms reduce to the reference code's per-batch ADE / FDE."""
    z = np.load(path)
    cs = val_inputs(z)
    nmax = int(z["w_Wi"].shape[0])
    S, F = len(cs), max(c[2] for c in cs)
    params = fs.G2KParams(**{k: torch.from_numpy(np.ascontiguousarray(z["w_" + k])).to(gpu)
                             for k in ("Wi", "Wii", "Wv", "bv", "Wr", "Wc", "Wo")})
    pos = np.stack([z[c[0] + "pos"] for c in cs])                         # [S, 8, Nmax, 2]
    vis = np.stack([z[c[0] + "vislet"] for c in cs])
    G = np.broadcast_to(z["G"], (S, 16, 8)).copy()
    tgt = np.stack([c[4] for c in cs])[:, None]                            # [S, 1, Nmax, 12, 2]
    mask = np.stack([c[5] for c in cs])
    t = lambda a, dt=torch.float32: torch.from_numpy(np.ascontiguousarray(a)).to(gpu, dt)  # noqa: E731
    out = fs.step_fused(params, t(pos), t(vis), t(G), t(tgt),
                        t([c[1] for c in cs], torch.int32), torch.zeros((S, 16, 128), device=gpu),
                        n_frames=t([c[2] for c in cs], torch.int32), ped_mask=t(mask, torch.uint8),
                        stride=0, targets_shared=True, frames=F, pred_layout=pred_layout)
    torch.cuda.synchronize()
    band = fs.pred_band(out.pred, pred_layout).cpu().numpy()
    for s, (p, n, nb, ref_band, _, _) in enumerate(cs):
        for f in range(nb):
            assert close(band[s, f, :, :n], ref_band) <= TOL
    check_batches(z, cs, out.metrics)


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p))
def test_get_mean_error_variant1_vs_reference_code(gpu, path):
    z = np.load(path)
    gs = [g for g in range(int(z["gm_count"]))
          if int(z[f"gm{g}_0_obs"]) == 8 and int(z[f"gm{g}_0_maxped"]) == z[f"gm{g}_true"].shape[0]]
    P = [z[f"gm{g}_true"].shape[0] for g in gs]
    nmax = max(P)
    S = len(gs)
    pred = np.zeros((S, 24, nmax), np.float32)
    tgt = np.zeros((S, nmax, 12, 2), np.float32)
    for s, g in enumerate(gs):
        pred[s, :, :P[s]] = z[f"gm{g}_pred"].reshape(24, P[s])
        tgt[s, :P[s]] = z[f"gm{g}_true"]
    out = fs.ade_fde(torch.from_numpy(pred).to(gpu), torch.from_numpy(tgt).to(gpu),
                     torch.tensor(P, dtype=torch.int32, device=gpu), variant=1).cpu().numpy()
    for s, g in enumerate(gs):
        q = f"gm{g}_0_"
        assert close(out[s, 0], z[q + "ade"]) <= TOL
        assert close(out[s, 1], z[q + "fde"]) <= TOL
        assert int(out[s, 2]) == int(z[q + "counter"])
