"""world_size-2 gloo test of the data-parallel path on CPU: each rank runs its
shard of scenes (the float64 oracle stands in for the GPU step here) and the
all-reduced metric sums equal the single-process sums."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from multimodaltraj_2_amd.dist import allreduce_grad, global_errors, reduce_metrics, shard_scenes


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene_metrics(S, lo, hi):
    from multimodaltraj_2_amd.synthetic import make_batch
    from oracle import g2k_ref as ref
    b = make_batch(S, 16, 64, F=4, seed=11)
    rng = np.random.default_rng(0)
    shapes = dict(Wi=(16, 16), Wii=(16, 8), Wv=(8, 18), bv=(16,), Wr=(8, 2), Wc=(24, 8), Wo=(8, 16))
    w = {k: rng.standard_normal(s) for k, s in shapes.items()}
    rows = []
    for s in range(lo, hi):
        _, _, m, _ = ref.scene_step(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s], b.n_active[s],
                                    b.h0[s], n_frames=b.F)
        rows.append(m)
    return torch.tensor(np.array(rows), dtype=torch.float64).reshape(-1, 8)


def _worker(rank, world, port, S, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_scenes(S, rank, world)
    tot = reduce_metrics(_scene_metrics(S, lo, hi))
    if rank == 0:
        q.put(tot.numpy())
    dist.destroy_process_group()


def test_shard_scenes_partition():
    for total in (0, 1, 7, 256, 1023):
        for world in (1, 2, 3, 8):
            spans = [shard_scenes(total, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_scenes(4, 2, 2)


def test_two_rank_gloo_metric_reduction():
    S, world = 6, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = _scene_metrics(S, 0, S).sum(dim=0).numpy()
    np.testing.assert_allclose(got, want, rtol=1e-12)
    ade, fde = global_errors(torch.tensor(got))
    assert np.isfinite(ade) and np.isfinite(fde)


def _scene_grads(S, lo, hi):
    """Flat [P + 2] train-mode buffer (gradient sums, loss, count) of scenes
    [lo, hi) from the float64 oracle (stands in for g2k_step_grad_f32)."""
    from multimodaltraj_2_amd.synthetic import make_batch
    from oracle import g2k_ref as ref
    b = make_batch(S, 16, 64, F=3, seed=12)
    rng = np.random.default_rng(0)
    shapes = dict(Wi=(16, 16), Wii=(16, 8), Wv=(8, 18), bv=(16,), Wr=(8, 2), Wc=(24, 8), Wo=(8, 16))
    w = {k: rng.standard_normal(s) for k, s in shapes.items()}
    flat = np.zeros(24 * 16 + 498)
    for s in range(lo, hi):
        loss, cnt, g = ref.scene_loss_grad(b.pos[s], b.vislet[s], b.G[s], w, b.targets[s],
                                           b.n_active[s], n_frames=b.F, lam=0.05)
        flat[:-2] += np.concatenate([g[k].reshape(-1) for k in ref.GRAD_ORDER])
        flat[-2] += loss
        flat[-1] += cnt
    return torch.tensor(flat, dtype=torch.float64)


def _grad_worker(rank, world, port, S, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_scenes(S, rank, world)
    g = allreduce_grad(_scene_grads(S, lo, hi))
    q.put((rank, g.numpy()))
    dist.destroy_process_group()


def test_two_rank_gloo_gradient_allreduce():
    """Train mode: each rank's shard gradient, summed by the one all-reduce,
    equals the whole-batch gradient on every rank (identical updates)."""
    S, world = 5, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_grad_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = _scene_grads(S, 0, S).numpy()
    for r in range(world):
        np.testing.assert_allclose(got[r], want, rtol=1e-12, atol=1e-12)


class _FakePlan:
    """Stands in for TrainPlan (the HIP launch) on CPU: its gradient buffer is
    the float64 oracle's [P + 2] for the rank's shard."""

    def __init__(self, grad, log):
        self.grad, self.log = grad, log

    def run(self, flat=None, ms=None, **kw):
        assert flat is None            # the collective structure never fuses the update
        self.log.append("gradient")
        return self.grad


def _structure_worker(rank, world, port, S, steps, q):
    from multimodaltraj_2_amd import train_step as tsm
    from oracle import g2k_ref as ref
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # collective=False across ranks would let the replicas drift: refused
    # before anything is bound
    try:
        tsm.TrainStep(None, None, None, None, None, None, None, collective=False)
        refused = False
    except ValueError:
        refused = True
    lo, hi = shard_scenes(S, rank, world)
    log = []
    P = _scene_grads(S, 0, 1).numel() - 2
    ts = object.__new__(tsm.TrainStep)            # no HIP library on CPU: the plans are fakes
    ts.flat = torch.linspace(-1, 1, P, dtype=torch.float64)
    ts.ms = torch.ones_like(ts.flat)
    ts.lr, ts.decay, ts.grad_clip = 0.005, 0.95, 10.0
    ts.group, ts.world, ts.collective = None, world, world > 1
    ts._layout = dict(stream=None)
    shard = _scene_grads(S, lo, hi)
    ts._slots = [_FakePlan(shard.clone(), log)]

    def fake_allreduce(buf, group=None, force=False):
        log.append("allreduce")
        return allreduce_grad(buf, group, force)

    def fake_update(flat, grad, *, lr, decay, grad_clip, ms=None, stream=None):
        log.append("update")
        p, m = ref.optimizer_update(flat.numpy(), ms.numpy(), grad[:-2].numpy(),
                                    float(grad[-1]), lr, decay, grad_clip)
        flat.copy_(torch.from_numpy(p))
        ms.copy_(torch.from_numpy(m))

    tsm.allreduce_grad, tsm.optimizer_update = fake_allreduce, fake_update
    for _ in range(steps):
        ts._slots[0].grad.copy_(shard)
        ts.run(0)
    q.put((rank, log, ts.flat.numpy(), ts.ms.numpy(), refused))
    dist.destroy_process_group()


def test_two_rank_gloo_train_step_structure():
    """TrainStep.run across ranks: per step gradient ->
    ONE all-reduce of the [P + 2] buffer -> update, in that order; every rank
    ends with the parameters one rank gets from the whole batch's gradient."""
    from oracle import g2k_ref as ref
    S, world, steps = 5, 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_structure_worker, args=(r, world, port, S, steps, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, rest) for r, *rest in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = _scene_grads(S, 0, S).numpy()
    flat = np.linspace(-1, 1, g.size - 2)
    ms = np.ones_like(flat)
    for _ in range(steps):
        flat, ms = ref.optimizer_update(flat, ms, g[:-2], float(g[-1]), 0.005, 0.95, 10.0)
    for r in range(world):
        log, f, m, refused = got[r]
        assert refused, "TrainStep(collective=False) in a 2-rank group must raise"
        assert log == ["gradient", "allreduce", "update"] * steps
        np.testing.assert_allclose(f, flat, rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(m, ms, rtol=1e-12, atol=1e-14)
