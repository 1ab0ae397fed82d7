"""GPU: the fused step's layout options (g2k_dims.flags, include/g2k_hip.h).

G2K_STEP_PRED_PED_MAJOR writes pred as [S, F, Nmax, L, 2] — the per-pedestrian
view train.py:254 transposes pred_path_band into — and only the active
pedestrians; G2K_STEP_TARGETS_SHARED reads one [S, 1, Nmax, L, 2] target set
for every frame (real-data scenes: the reference feeds a batch's targets to
every frame of its loop).  Both must give bit-identical results to the
default layouts (same arithmetic, other addresses), forward and train mode;
the oracle parity of the default layouts is in test_step_gpu / test_train_gpu."""
import ctypes

import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import _lib
from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd import train_step as ts
from multimodaltraj_2_amd.synthetic import make_batch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("Nmax,H", [(32, 128), (64, 256), (256, 256), (20, 64)])
def test_ped_major_pred_equals_band(gpu, Nmax, H):
    b = make_batch(24, Nmax, H, seed=5)
    t = b.to_device(gpu)
    params = fs.init_params(Nmax, seed=0, device=gpu)
    ref = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    out = fs.StepOutputs(pred=torch.full(fs.pred_shape(b.S, b.F, Nmax, "ped"), float("nan"), device=gpu),
                         h=torch.empty_like(t["h0"]), metrics=torch.empty((b.S, 8), device=gpu))
    got = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                        pred_layout="ped", out=out)
    torch.cuda.synchronize()
    band = fs.pred_band(got.pred, "ped").cpu().numpy()
    want = ref.pred.cpu().numpy()
    for s in range(b.S):
        n = int(b.n_active[s])
        np.testing.assert_array_equal(band[s, :, :, :n], want[s, :, :, :n])
        assert np.isnan(got.pred[s, :, n:].cpu().numpy()).all()      # inactive: not written
    np.testing.assert_array_equal(got.h.cpu().numpy(), ref.h.cpu().numpy())
    np.testing.assert_array_equal(got.metrics.cpu().numpy(), ref.metrics.cpu().numpy())


def _shared_batch(gpu, S=32, Nmax=32, H=128, F=9):
    """Stride-0 scenes whose targets are the same in every frame."""
    b = make_batch(S, Nmax, H, F=F, seed=9)
    t = b.to_device(gpu)
    t["pos"] = t["pos"][:, :8].contiguous()
    t["targets1"] = t["targets"][:, :1].contiguous()
    t["targets"] = t["targets1"].expand(-1, F, -1, -1, -1).contiguous()
    t["n_frames"] = torch.from_numpy(np.random.default_rng(2).integers(0, F + 1, S).astype(np.int32)).to(gpu)
    return b, t, F


@pytest.mark.parametrize("split", [0, 2])
def test_shared_targets_equal_replicated(gpu, split):
    """split 2: both launches take the general path (same arithmetic, other
    addresses: bit-identical); split 0: the shared launch's automatic split
    is 1 and it takes the loop-invariant path (pred, h bit-identical; the
    metric sums n_frames x one frame's terms, within 1e-6)."""
    b, t, F = _shared_batch(gpu)
    params = fs.init_params(32, seed=0, device=gpu)
    kw = dict(n_frames=t["n_frames"], stride=0, split=split)
    ref = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                        **kw)
    got = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets1"], t["n_active"], t["h0"],
                        targets_shared=True, frames=F, **kw)
    torch.cuda.synchronize()
    for k in ("pred", "h"):
        np.testing.assert_array_equal(getattr(got, k).cpu().numpy(), getattr(ref, k).cpu().numpy())
    gm, rm = got.metrics.cpu().numpy(), ref.metrics.cpu().numpy()
    if split:
        np.testing.assert_array_equal(gm, rm)
    else:
        assert np.abs(gm - rm).max() <= 1e-6 * max(1.0, np.abs(rm).max())
        np.testing.assert_array_equal(gm[:, [1, 5]], rm[:, [1, 5]])


@pytest.mark.parametrize("layout,coresident", [("band", False), ("ped", False), ("ped", True)])
def test_invariant_frames_equal_general_path(gpu, layout, coresident):
    """Stride 0 with shared targets and one workgroup per scene: every frame
    has the same inputs, and the forward forms one head and one set of tiles
    per chunk and replicates them (g2k_scene.hip frames_invariant).  Against
    the general path on the same frames (replicated targets): pred, h, attn
    and cost bit-identical (the same arithmetic per frame); the metric sums
    within 1e-6 relative (n_frames x one frame's terms instead of a sum over
    frames).  F = 40: two chunks of frames (kSceneChunk = 32)."""
    S, F = 24, 40
    b = make_batch(S, 32, 128, F=F, seed=11)
    t = b.to_device(gpu)
    pos = t["pos"][:, :8].contiguous()
    tgt1 = t["targets"][:, :1].contiguous()
    nf = torch.from_numpy(np.random.default_rng(4).integers(0, F + 1, S).astype(np.int32)).to(gpu)
    nf[0], nf[1] = F, 33                                   # both chunks, a 1-frame second chunk
    params = fs.init_params(32, seed=0, device=gpu)
    kw = dict(n_frames=nf, stride=0, want_attn=True, pred_layout=layout, split=1)
    ref = fs.step_fused(params, pos, t["vislet"], t["G"], tgt1.expand(-1, F, -1, -1, -1).contiguous(),
                        t["n_active"], t["h0"], **kw)
    got = fs.step_fused(params, pos, t["vislet"], t["G"], tgt1, t["n_active"], t["h0"],
                        targets_shared=True, frames=F, coresident=coresident, **kw)
    torch.cuda.synchronize()
    nfh = nf.cpu().numpy()
    for s in range(S):
        n, f = int(b.n_active[s]), int(nfh[s])
        gp, rp = fs.pred_band(got.pred, layout)[s, :f, :, :n], fs.pred_band(ref.pred, layout)[s, :f, :, :n]
        assert torch.equal(gp, rp), s
        assert torch.equal(got.attn[s, :f], ref.attn[s, :f]) and torch.equal(got.cost[s, :f], ref.cost[s, :f]), s
    assert torch.equal(got.h, ref.h)
    gm, rm = got.metrics.cpu().numpy(), ref.metrics.cpu().numpy()
    assert np.abs(gm - rm).max() <= 1e-6 * max(1.0, np.abs(rm).max())
    np.testing.assert_array_equal(gm[:, 1], rm[:, 1])      # the pair counts
    np.testing.assert_array_equal(gm[:, 5], rm[:, 5])      # frames


@pytest.mark.parametrize("layout,shared,split", [("ped", False, 0), ("band", True, 2),
                                                  ("ped", True, 2), ("ped", True, 0)])
def test_train_step_layouts_equal_default(gpu, layout, shared, split):
    """Same arithmetic, other addresses: bit-identical — except shared targets
    at the automatic split (1: the loop-invariant train path, one frame's
    gradient terms with weight n_frames), whose gradient is checked within
    1e-5 of the general path's (max |difference| against max |entry|), with
    the same pair count and bit-identical predictions."""
    b, t, F = _shared_batch(gpu)
    kw = dict(n_frames=t["n_frames"], stride=0, split=split)
    grads, preds = [], []
    for lay, sh in (("band", False), (layout, shared)):
        params = fs.init_params(32, seed=0, device=gpu)
        tgt = t["targets1"] if sh else t["targets"]
        tp = ts.TrainPlan(params, t["pos"], t["vislet"], t["G"], tgt, t["n_active"], t["h0"],
                          pred_layout=lay, targets_shared=sh, frames=F if sh else None, **kw)
        g = tp.run().clone()
        gp = ts.GradPlan(params, t["pos"], t["vislet"], t["G"], tgt, t["n_active"],
                         targets_shared=sh, frames=F if sh else None, **kw).run()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(g.cpu().numpy(), gp.cpu().numpy())
        grads.append(g.cpu().numpy())
        preds.append(fs.pred_band(tp.out.pred, lay).cpu().numpy())
    if shared and not split:
        g0, g1 = grads
        assert np.abs(g0 - g1).max() <= 1e-5 * np.abs(g0).max()
        assert g0[-1] == g1[-1]                                # the pair count
    else:
        np.testing.assert_array_equal(grads[0], grads[1])
    for s in range(b.S):
        n = int(b.n_active[s])
        np.testing.assert_array_equal(preds[0][s, :, :, :n], preds[1][s, :, :, :n])


def test_flags_rejected_where_unsupported(gpu):
    lib = _lib.load()
    d = _lib.G2KDims(1, 1, 8, 12, 16, 64, 8, 8, 0, _lib.STEP_PRED_PED_MAJOR)
    x = torch.zeros(4096, device=gpu)
    rc = lib.g2k_ade_fde_f32(ctypes.byref(d), x.data_ptr(), x.data_ptr(), x.data_ptr(), None, None,
                             0, x.data_ptr(), None)
    assert rc == -4 and b"flags" in lib.g2k_last_error()
    d.flags = 16                                      # no such flag
    assert lib.g2k_step_workspace_bytes(ctypes.byref(d)) == -1
    # G2K_STEP_CORESIDENT is a forward-step option: the train entry points reject it
    d.flags = _lib.STEP_CORESIDENT
    assert lib.g2k_step_workspace_bytes(ctypes.byref(d)) == 0
    assert lib.g2k_train_workspace_bytes(ctypes.byref(d)) == -1
    assert lib.g2k_grad_size(ctypes.byref(d)) == -1
