"""GPU parity: the fused HIP step vs the float64 oracle (oracle/g2k_ref.py).
Tolerances (written here): pred and the metric sums
|got - ref| <= 1e-4 * max(1, |ref|); the hidden state h (entries ~1/H) is held
relatively, |got - ref| <= 1e-5 * |ref| + 1e-8 (close_h)."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd.synthetic import make_batch
from oracle import g2k_ref as ref
from multimodaltraj_2_amd.synthetic import CONFIGS
from tests.conftest import close, close_h

TOL = 1e-4
pytestmark = pytest.mark.gpu


def run_both(S, Nmax, H, F=20, seed=1, n_active=None, h0_scale=0.0, ped_mask=None,
             n_frames=None, device=None, lam=fs.LAMBDA):
    b = make_batch(S, Nmax, H, F=F, seed=seed, n_active=n_active, h0_scale=h0_scale)
    params = fs.init_params(Nmax, seed=0, device=device)
    t = b.to_device(device)
    pm = None if ped_mask is None else torch.from_numpy(ped_mask.astype(np.uint8)).to(device)
    nfr = None if n_frames is None else torch.from_numpy(np.asarray(n_frames, np.int32)).to(device)
    out = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                        t["h0"], n_frames=nfr, ped_mask=pm, stride=1, want_attn=True, lam=lam)
    torch.cuda.synchronize()
    w = params.numpy()
    res = []
    for s in range(S):
        nf = F if n_frames is None else int(n_frames[s])
        pr, h, m, ex = ref.scene_step(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s],
                                      b.n_active[s], b.h0[s], n_frames=nf, stride=1,
                                      ped_mask=None if ped_mask is None else ped_mask[s],
                                      keep=True, lam=lam)
        res.append((pr, h, m, ex))
    return b, out, res


@pytest.mark.parametrize("S,Nmax,H", [(4, 32, 128), (3, 64, 256), (2, 8, 64), (2, 256, 128)])
def test_step_matches_oracle(gpu, S, Nmax, H):
    b, out, res = run_both(S, Nmax, H, device=gpu)
    pred = out.pred.cpu().numpy()
    hh = out.h.cpu().numpy()
    met = out.metrics.cpu().numpy()
    attn = out.attn.cpu().numpy()
    cost = out.cost.cpu().numpy()
    for s in range(S):
        n = int(b.n_active[s])
        pr, h, m, ex = res[s]
        # pred_path_band [2, L, n] per frame == our [2L, Nmax] rows
        got = pred[s, :, :, :n].reshape(pred.shape[1], 2, 12, n)
        assert close(got, pr) <= TOL
        assert np.all(pred[s, :, :, n:] == 0)
        # attn/cost are intermediates (not outputs of the reference path):
        # A = g @ (E*Rm) cancels heavily at N = 256, so it is held to the
        # normwise bound |dA| <= 1e-4 * max(1, max|A|) (fp32 condition).
        A_ref = np.stack(ex["A"])
        assert np.abs(attn[s] - A_ref).max() <= TOL * max(1.0, np.abs(A_ref).max())
        assert close(cost[s], np.stack(ex["cost"])) <= TOL
        assert close_h(hh[s], h)
        assert close(met[s, :6], m[:6]) <= TOL


def test_step_large_logits(gpu):
    """lambda = 0.1 puts |A| up to ~160 with column spreads > 87, where
    exp(A - column max) underflows: the running-max fallback of the As step
    (train.py:240) must take over (the float64 oracle is exact there)."""
    b, out, res = run_both(3, 32, 64, F=12, device=gpu, lam=0.1)
    hh = out.h.cpu().numpy()
    attn = out.attn.cpu().numpy()
    pred = out.pred.cpu().numpy()
    for s in range(3):
        n = int(b.n_active[s])
        pr, h, m, ex = res[s]
        A_ref = np.stack(ex["A"])
        assert np.abs(A_ref).max() > 87.0
        assert np.abs(attn[s] - A_ref).max() <= TOL * max(1.0, np.abs(A_ref).max())
        assert close(pred[s, :, :, :n].reshape(12, 2, 12, n), pr) <= TOL
        assert close_h(hh[s], h)


def test_step_nonzero_h0_and_masks(gpu):
    S, Nmax = 3, 32
    mask = np.ones((S, Nmax), bool)
    mask[0, ::3] = False
    b, out, res = run_both(S, Nmax, 128, h0_scale=3.0, ped_mask=mask, n_frames=[20, 7, 0],
                           device=gpu)
    met = out.metrics.cpu().numpy()
    hh = out.h.cpu().numpy()
    pred = out.pred.cpu().numpy()
    for s in range(S):
        pr, h, m, ex = res[s]
        n = int(b.n_active[s])
        nf = pr.shape[0]
        assert close(pred[s, :nf, :, :n].reshape(nf, 2, 12, n), pr) <= TOL
        assert np.all(pred[s, nf:] == 0)
        assert close_h(hh[s], h)
        assert close(met[s, :6], m[:6]) <= TOL


@pytest.mark.parametrize("Nmax", [30, 64])
def test_step_masks_byte_and_dword_rows(gpu, Nmax):
    """ped_mask rows read per byte (Nmax % 4 != 0) and per dword (ballot
    spread), with pedestrians masked at every residue mod 4 and past a tile
    boundary; columns of the written tiles past n_active are 0."""
    S = 3
    mask = np.ones((S, Nmax), bool)
    mask[0, 1::4] = False
    mask[1, 2::5] = False
    mask[2, 16:20] = False
    b, out, res = run_both(S, Nmax, 128, ped_mask=mask, n_frames=[20, 13, 20], device=gpu)
    met = out.metrics.cpu().numpy()
    pred = out.pred.cpu().numpy()
    for s in range(S):
        pr, h, m, ex = res[s]
        n = int(b.n_active[s])
        nf = pr.shape[0]
        assert close(pred[s, :nf, :, :n].reshape(nf, 2, 12, n), pr) <= TOL
        assert np.all(pred[s, :, :, n:] == 0)
        assert close(met[s, :6], m[:6]) <= TOL


def test_step_deterministic(gpu):
    b = make_batch(8, 32, 128, seed=5)
    params = fs.init_params(32, seed=0, device=gpu)
    t = b.to_device(gpu)
    o1 = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    o2 = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    torch.cuda.synchronize()
    assert torch.equal(o1.pred, o2.pred)
    assert torch.equal(o1.h, o2.h)
    assert torch.equal(o1.metrics, o2.metrics)


def test_mcr_forward_matches_oracle(gpu):
    rng = np.random.default_rng(3)
    S, Nmax = 5, 32
    params = fs.init_params(Nmax, seed=0, device=gpu)
    w = params.numpy()
    X = rng.standard_normal((S, 18, 16)).astype(np.float32)
    Rel = rng.standard_normal((S, 2, 16)).astype(np.float32)
    G = rng.standard_normal((S, 16, 8)).astype(np.float32)
    nact = np.array([32, 1, 17, 8, 30], np.int32)
    A, C, P = fs.mcr_forward(params, torch.from_numpy(X).to(gpu), torch.from_numpy(Rel).to(gpu),
                             torch.from_numpy(G).to(gpu), torch.from_numpy(nact).to(gpu))
    torch.cuda.synchronize()
    A, C, P = A.cpu().numpy(), C.cpu().numpy(), P.cpu().numpy()
    for s in range(S):
        n = nact[s]
        o = ref.mcr_forward(X[s].astype(np.float64), Rel[s], G[s], w["Wv"], w["bv"], w["Wr"],
                            w["Wc"], w["Wo"][:, :n], 5e-4)
        assert close(A[s], o["attn"]) <= TOL
        assert close(C[s], o["cost"]) <= TOL
        assert close(P[s][:, :n].reshape(2, 12, n), o["pred_path_band"]) <= TOL


def test_recurrence_matches_oracle(gpu):
    rng = np.random.default_rng(4)
    S, F, H = 3, 6, 128
    A = (2.0 * rng.standard_normal((S, F, 16, 16))).astype(np.float32)
    A[0, 0, 3, :] += 60.0      # large logits: exercises the running-max column pass
    h0 = rng.standard_normal((S, 16, H)).astype(np.float32)
    h = torch.from_numpy(h0).to(gpu)
    fs.frame_recurrence(torch.from_numpy(A).to(gpu), h)
    torch.cuda.synchronize()
    got = h.cpu().numpy()
    for s in range(S):
        hr = h0[s].astype(np.float64)
        for f in range(F):
            hr = ref.recurrence_step(A[s, f].astype(np.float64), hr)
        assert close_h(got[s], hr)


def test_ade_fde_variants(gpu):
    rng = np.random.default_rng(6)
    S, F, Nmax = 3, 5, 16
    pred = rng.standard_normal((S, F, 24, Nmax)).astype(np.float32)
    tgt = rng.standard_normal((S, F, Nmax, 12, 2)).astype(np.float32)
    nact = np.array([16, 3, 9], np.int32)
    out = fs.ade_fde(torch.from_numpy(pred).to(gpu), torch.from_numpy(tgt).to(gpu),
                     torch.from_numpy(nact).to(gpu)).cpu().numpy()
    for s in range(S):
        m = np.zeros(6)
        for f in range(F):
            P_ = pred[s, f].reshape(2, 12, Nmax).transpose(2, 1, 0).astype(np.float64)
            for i in range(nact[s]):
                a, e = ref.validation_errors(P_[i], tgt[s, f, i])
                d = P_[i] - tgt[s, f, i]
                m += [a, 1, e @ e, np.mean(np.linalg.norm(d, axis=1)), np.linalg.norm(e), 0]
        m[5] = F
        assert close(out[s, :6], m) <= TOL
    # variant 1: sample.py get_mean_error
    p1 = pred[:, 0]
    t1 = tgt[:, 0]
    out1 = fs.ade_fde(torch.from_numpy(np.ascontiguousarray(p1)).to(gpu),
                      torch.from_numpy(np.ascontiguousarray(t1)).to(gpu),
                      torch.from_numpy(nact).to(gpu), variant=1).cpu().numpy()
    for s in range(S):
        n = nact[s]
        complete = p1[s][:, :n].reshape(2, 12, n).transpose(2, 1, 0)
        ade, fde, cnt = ref.get_mean_error(complete, t1[s][:n], 8, n)
        assert close(out1[s, :3], [ade, fde, cnt]) <= TOL


def _check_all(b, out, res, S):
    pred = out.pred.cpu().numpy()
    hh = out.h.cpu().numpy()
    met = out.metrics.cpu().numpy()
    for s in range(S):
        n = int(b.n_active[s])
        pr, h, m, ex = res[s]
        nf = pr.shape[0]
        assert close(pred[s, :nf, :, :n].reshape(nf, 2, 12, n), pr) <= TOL
        assert np.all(pred[s, :, :, n:] == 0)
        assert close_h(hh[s], h)
        assert close(met[s, :6], m[:6]) <= TOL


@pytest.mark.parametrize("S,Nmax,H,F", [(3, 7, 64, 20), (2, 32, 128, 40), (2, 30, 64, 33)])
def test_step_fallbacks_and_chunks(gpu, S, Nmax, H, F):
    """Odd Nmax and Nmax = 30 (odd 16-B slots per row) under the default
    4-byte staging; F beyond the
    32-frame chunk exercises the chunked prologue (fb > 0) and the recurrence
    waves' heads of a later chunk; Nmax = 30 has an odd number of 16-B slots
    per position row."""
    b, out, res = run_both(S, Nmax, H, F=F, device=gpu)
    _check_all(b, out, res, S)


# BASELINE.json configs at their own benchmark shapes (bench.py rank 0
# batch): every 16th scene in full (pred, h, metrics) and the metric sums
# over all scenes.  cfg 5 (Nmax 256, H 256) is the LDS-chunked layout.
CFG = [("eth_hotel_synth", 256), ("eth_ucy_loo_kfold4", 128), ("relational_attn_h256", 256),
       ("dense_crowd", 128)]


@pytest.mark.parametrize("coresident", [False, True])
@pytest.mark.parametrize("name,S", CFG)
def test_config_shape_matches_oracle(gpu, name, S, coresident):
    """coresident: G2K_STEP_CORESIDENT (8-wave workgroups, two per CU; the
    usual geometry where the LDS does not fit twice, dense_crowd)."""
    c = CONFIGS[name]
    Nmax, H = c["Nmax"], c["H"]
    b = make_batch(S, Nmax, H, seed=1)
    params = fs.init_params(Nmax, seed=0, device=gpu)
    t = b.to_device(gpu)
    out = fs.step_fused(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                        t["h0"], coresident=coresident)
    torch.cuda.synchronize()
    pred, hh, met = out.pred.cpu().numpy(), out.h.cpu().numpy(), out.metrics.cpu().numpy()
    w = params.numpy()
    tot = np.zeros(6)
    for s in range(S):
        pr, h, m, _ = ref.scene_step(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s],
                                     b.n_active[s], b.h0[s], n_frames=b.F)
        tot += m[:6]
        if s % 16 == 0 or s == S - 1:
            n = int(b.n_active[s])
            assert close(pred[s, :, :, :n].reshape(b.F, 2, 12, n), pr) <= TOL, s
            assert close_h(hh[s], h), s
            assert close(met[s, :6], m[:6]) <= TOL, s
    assert close(met[:, :6].astype(np.float64).sum(axis=0), tot) <= TOL


def test_step_h512_long_chain_margin(gpu):
    """The split-f16 recurrence product at its widest (H = 512: row sums Z ~
    H, the A operand ~ 128 As log2(e) / Z smallest) over a long chain (F = 100
    frames, nonzero h0): h stays inside close_h's 1e-5 relative bound
    (DESIGN.md §6a "Recurrence numerics": worst-case ~6e-6 per frame at H = 512,
    the rounding errors do not compound across frames because every frame
    renormalises).  The measured margin is printed."""
    b, out, res = run_both(2, 32, 512, F=100, device=gpu, h0_scale=1.0)
    hh = out.h.cpu().numpy()
    worst = 0.0
    for s in range(2):
        h = res[s][1]
        worst = max(worst, float(np.max(np.abs(hh[s] - h) / (np.abs(h) + 1e-3 / 512))))
        assert close_h(hh[s], h)
    print(f"H=512 F=100: max |dh| / |h| = {worst:.2e} (bound 1e-5)")


def test_frame_embed_matches_oracle(gpu):
    """g2k_frame_embed_f32 (a2-a4 alone) vs oracle window_norms / input_embed /
    vislet_embed for every frame of a stride-1 window (Nmax 64, n from 1)."""
    S, Nmax, F = 3, 64, 6
    b = make_batch(S, Nmax, 128, F=F, seed=9, n_active=np.array([64, 1, 23], np.int32))
    params = fs.init_params(Nmax, seed=0, device=gpu)
    t = b.to_device(gpu)
    X, Rel = fs.frame_embed(params, t["pos"], t["vislet"], t["n_active"], F, stride=1)
    torch.cuda.synchronize()
    X, Rel = X.cpu().numpy(), Rel.cpu().numpy()
    w = params.numpy()
    for s in range(S):
        n = int(b.n_active[s])
        Wi = w["Wi"][:n].astype(np.float64)
        Ve, R = ref.vislet_embed(b.vislet[s][:, :n].astype(np.float64), Wi)
        assert close(Rel[s], R) <= TOL
        for f in range(F):
            Bv = ref.window_norms(b.pos[s][f:f + 8, :n].astype(np.float64))
            X0 = ref.input_embed(Bv, Wi, w["Wii"].astype(np.float64))
            assert close(X[s, f], np.concatenate((X0, Ve), axis=0)) <= TOL


@pytest.mark.parametrize("name,S", [("eth_hotel_synth", 256), ("eth_ucy_loo_kfold4", 128)])
def test_coresident_launches_in_flight(gpu, name, S):
    """G2K_STEP_CORESIDENT launches of 8 independent batches round-robin over
    4 streams (bench.py's timed pattern, two workgroups per CU) compute, bit
    for bit, what each launch computes alone; pred and h are also bit-identical
    to the one-workgroup-per-CU geometry (same per-frame arithmetic; the metric
    sums add the producers' partials in another grouping: 1e-4)."""
    c = CONFIGS[name]
    Nmax, H = c["Nmax"], c["H"]
    assert fs.step_coresidency(S, 20, H, Nmax, 27, 1, True) == 2
    params = fs.init_params(Nmax, seed=0, device=gpu)
    streams = [torch.cuda.Stream(device=gpu) for _ in range(4)]
    plans, alone = [], []
    for k in range(8):
        t = make_batch(S, Nmax, H, seed=10 + k).to_device(gpu)
        args = (params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
        plans.append(fs.StepPlan(*args, stream=streams[k % 4], pred_layout="ped", coresident=True))
        alone.append(fs.step_fused(*args, pred_layout="ped", coresident=True))
        base = fs.step_fused(*args, pred_layout="ped")
        torch.cuda.synchronize()
        assert torch.equal(alone[-1].pred, base.pred) and torch.equal(alone[-1].h, base.h)
        assert close(alone[-1].metrics.cpu().numpy(), base.metrics.cpu().numpy()) <= TOL
    torch.cuda.synchronize()
    for _ in range(3):
        for p in plans:
            p.run()
    torch.cuda.synchronize()
    for p, a in zip(plans, alone):
        assert torch.equal(p.out.pred, a.pred)
        assert torch.equal(p.out.h, a.h)
        assert torch.equal(p.out.metrics, a.metrics)


@pytest.mark.parametrize("coresident", [False, True])
def test_step_stride2_matches_oracle(gpu, coresident):
    """Window stride 2 (frame f's window starts at row 2 f): 46 window rows,
    so the staging has more tasks than a co-resident workgroup has producer
    waves (4 V / VG tiles, K1 / K2 and the padded operands' constants over 4
    producers: the task loop wraps), and the frame heads read their window
    rows at 2 f + k."""
    S, Nmax, H, F = 3, 32, 128, 20
    b = make_batch(S, Nmax, H, F=2 * F - 1, seed=5, h0_scale=1.0)   # W = 2 (F - 1) + 8 rows
    tg = np.ascontiguousarray(b.targets[:, ::2])                    # any F target sets
    params = fs.init_params(Nmax, seed=0, device=gpu)
    t = b.to_device(gpu)
    out = fs.step_fused(params, t["pos"], t["vislet"], t["G"], torch.from_numpy(tg).to(gpu),
                        t["n_active"], t["h0"], stride=2, coresident=coresident)
    torch.cuda.synchronize()
    pred, hh, met = out.pred.cpu().numpy(), out.h.cpu().numpy(), out.metrics.cpu().numpy()
    w = params.numpy()
    for s in range(S):
        pr, h, m, _ = ref.scene_step(b.pos[s], b.vislet[s], b.G[s], w, tg[s], b.n_active[s],
                                     b.h0[s], n_frames=F, stride=2)
        n = int(b.n_active[s])
        assert close(pred[s, :, :, :n].reshape(F, 2, 12, n), pr) <= TOL, s
        assert close_h(hh[s], h), s
        assert close(met[s, :6], m[:6]) <= TOL, s
