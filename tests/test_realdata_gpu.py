"""GPU: config 3's workload on real data — 128 DISTINCT ETH/UCY scenes (the
reference's data files, tests/golden/data_*.npz; multimodaltraj_2_amd/realdata.py:
sample.py's scene per frame pointer, planned natively and expanded by
g2k_scene_gather_f32) in ONE [S, ...] launch of g2k_step_fused_f32 and
g2k_step_grad_f32, EVERY scene checked against the float64 oracle.
Tolerances as tests/test_step_gpu.py / tests/test_train_gpu.py."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd import realdata as rd
from multimodaltraj_2_amd import train_step as ts
from oracle import g2k_ref as ref
from tests.conftest import close, close_h
from tests.test_realdata import RAW

pytestmark = pytest.mark.gpu
TOL = 1e-4
H = 128


@pytest.fixture(scope="module")
def plan():
    return rd.plan_scenes(128, RAW)


@pytest.fixture(scope="module")
def dev_batch(gpu, plan):
    t = plan.to_device(gpu)
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)
    t["G"] = torch.from_numpy(rng.standard_normal((plan.S, 16, 8)).astype(np.float32)).to(gpu)
    t["h0"] = torch.zeros((plan.S, 16, H), device=gpu)
    return t


def test_device_gather_equals_host_expansion(plan, dev_batch):
    h = plan.host()
    for k in ("pos", "vislet", "targets", "ped_mask", "n_active", "n_frames"):
        np.testing.assert_array_equal(dev_batch[k].cpu().numpy(), h[k], err_msg=k)


@pytest.mark.parametrize("shared", [False, True])
def test_every_real_scene_matches_oracle(gpu, plan, dev_batch, shared):
    """shared: one target set per scene (G2K_STEP_TARGETS_SHARED) and one
    co-resident workgroup per scene — bench.py's real-data launch, which runs
    the loop-invariant forward (stride 0: one head and one set of tiles per
    chunk, replicated over the frames; g2k_scene.hip frames_invariant)."""
    t = dev_batch
    Nmax = plan.Nmax
    params = fs.init_params(Nmax, seed=0, device=gpu)
    tgt = t["targets"][:, :1].contiguous() if shared else t["targets"]
    out = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], tgt, t["n_active"], t["h0"],
                      n_frames=t["n_frames"], ped_mask=t["ped_mask"], stride=0,
                      targets_shared=shared, frames=int(t["targets"].shape[1]) if shared else None,
                      coresident=shared).run()
    torch.cuda.synchronize()
    h = plan.host()
    G = t["G"].cpu().numpy()
    w = params.numpy()
    pred, hh, met = out.pred.cpu().numpy(), out.h.cpu().numpy(), out.metrics.cpu().numpy()
    for s in range(plan.S):
        n, nf = int(plan.n_active[s]), int(plan.n_frames[s])
        pr, h_ref, m, _ = ref.scene_step(h["pos"][s], h["vislet"][s], G[s], w, h["targets"][s], n,
                                         np.zeros((16, H), np.float32), n_frames=nf, stride=0,
                                         ped_mask=h["ped_mask"][s].astype(bool))
        assert close(pred[s, :nf, :, :n].reshape(nf, 2, 12, n), pr) <= TOL, s
        assert close_h(hh[s], h_ref), s
        assert close(met[s, :6], m[:6]) <= TOL, s


@pytest.mark.parametrize("shared", [False, True])
def test_real_launch_gradient_matches_oracle(gpu, plan, dev_batch, shared):
    """shared: one target set per scene — the automatic split is 1 and the
    gradient takes the loop-invariant train path (one frame's terms with
    weight n_frames, g2k_scene.hip frames_invariant)."""
    S = 32
    Nmax = plan.Nmax
    params = fs.init_params(Nmax, seed=0, device=gpu)
    t = {k: (v[:S] if isinstance(v, torch.Tensor) else v) for k, v in dev_batch.items()}
    tgt = t["targets"][:, :1].contiguous() if shared else t["targets"]
    gp = ts.GradPlan(params, t["pos"], t["vislet"], t["G"], tgt, t["n_active"],
                     n_frames=t["n_frames"], ped_mask=t["ped_mask"], stride=0,
                     targets_shared=shared, frames=int(t["targets"].shape[1]) if shared else None)
    g = gp.run().double().cpu().numpy()
    h = plan.host()
    G = dev_batch["G"].cpu().numpy()
    w = params.numpy()
    loss, cnt, R = 0.0, 0, None
    for s in range(S):
        l_, c_, r_ = ref.scene_loss_grad(h["pos"][s], h["vislet"][s], G[s], w, h["targets"][s],
                                         int(plan.n_active[s]), n_frames=int(plan.n_frames[s]),
                                         stride=0, ped_mask=h["ped_mask"][s].astype(bool))
        loss += l_
        cnt += c_
        R = r_ if R is None else {k: R[k] + r_[k] for k in R}
    P = ts.grad_size(Nmax)
    off = 0
    for k in ref.GRAD_ORDER:
        r = R[k].reshape(-1)
        got = g[off:off + r.size]
        off += r.size
        if k == "Wr":
            assert np.all(got == 0)
        else:
            assert np.abs(got - r).max() <= TOL * max(np.abs(r).max(), 1e-30), k
    assert off == P
    assert abs(g[P] - loss) <= TOL * loss and g[P + 1] == cnt


def test_1024_scene_batch_built_fast(gpu):
    """A 1024-scene real batch, planned natively and gathered on the device,
    in well under a second (the walk of round 2 took 83 s)."""
    import time
    srcs = [rd.SceneSource(n, RAW[n]) for n in RAW]
    t0 = time.perf_counter()
    p = rd.plan_scenes(1024, RAW, sources=srcs)
    t = p.to_device(gpu)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert t["targets"].shape[0] == 1024
    print(f"1024 real scenes planned + gathered in {dt * 1e3:.1f} ms")
    assert dt < 0.5
