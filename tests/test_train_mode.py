"""--mode train through the entry point's loop (multimodaltraj_2_amd/train.py
train_mode) on CPU: world_size-2 gloo ranks, each taking its contiguous shard
of every global step of real scenes (realdata plans of the k-fold-4 datasets),
ONE all-reduce of the flat [P + 2] buffer per step, the same update on every
rank.  The float64 oracle stands in for the HIP step (OracleStepper: the
gradient of oracle.scene_loss_grad, the update of oracle.optimizer_update);
the GPU stepper is checked against this one in tests/test_train_mode_gpu.py.
After k steps the parameters are identical on both ranks and equal (to float64
rounding of the summation order) to the one-rank run over the union of the
shards."""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd import realdata as rd
from multimodaltraj_2_amd import train as tr

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
GRAD_ORDER = ("Wi", "Wii", "Wv", "bv", "Wr", "Wc", "Wo")


def _args(batch=4, epochs=2):
    from multimodaltraj_2_amd.argParser import ArgsParser
    a = ArgsParser().parser.parse_args([])
    a.train_batch, a.num_epochs, a.rnn_size = batch, epochs, 64
    return a


def small_plan(S=8):
    raw = {n: np.load(os.path.join(GOLDEN, f"data_{n}.npz"))["raw_data"]
           for n in rd.fold_datasets(4)}
    return rd.plan_scenes(S, raw, nmax=16)


class OracleStepper:
    """train_mode's stepper interface on the float64 oracle (test only)."""

    def __init__(self, args, plan, shard_idx, device, steps):
        from oracle import g2k_ref as ref
        self.ref, self.args = ref, args
        self.h = tr.plan_subset(plan, shard_idx).host()
        self.S = len(shard_idx)
        self.per = self.S // steps
        self.G = tr.context_G(args.seed, self.S)
        p = fs.init_params(plan.Nmax, seed=args.seed).numpy()
        self.shapes = {k: p[k].shape for k in GRAD_ORDER}
        self.flat = np.concatenate([p[k].astype(np.float64).reshape(-1) for k in GRAD_ORDER])
        self.ms = np.ones_like(self.flat)

    def _weights(self):
        out, o = {}, 0
        for k in GRAD_ORDER:
            n = int(np.prod(self.shapes[k]))
            out[k] = self.flat[o:o + n].reshape(self.shapes[k])
            o += n
        return out

    def grad(self, k):
        w, h = self._weights(), self.h
        buf = np.zeros(self.flat.size + 2)
        for s in range(k * self.per, (k + 1) * self.per):
            loss, cnt, g = self.ref.scene_loss_grad(
                h["pos"][s], h["vislet"][s], self.G[s], w, h["targets"][s], int(h["n_active"][s]),
                n_frames=int(h["n_frames"][s]), stride=0, lam=self.args.lambda_param,
                ped_mask=h["ped_mask"][s].astype(bool))
            buf[:-2] += np.concatenate([g[key].reshape(-1) for key in GRAD_ORDER])
            buf[-2] += loss
            buf[-1] += cnt
        return torch.from_numpy(buf)

    def apply(self, g):
        g = g.numpy()
        a = self.args
        self.flat, self.ms = self.ref.optimizer_update(self.flat, self.ms, g[:-2], g[-1],
                                                       a.learning_rate, a.decay_rate, a.grad_clip)

    def fused(self, k):
        g = self.grad(k)
        self.apply(g)
        return g

    def params(self):
        return self.flat.copy()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class HostReads:
    """Counts host reads of tensors (cpu / numpy / item / tolist / float)
    issued from train.train_mode itself — the entry point's loop, not the
    stepper (the oracle stand-in computes on the host by design)."""

    NAMES = ("cpu", "numpy", "item", "tolist", "__float__")

    def __init__(self):
        self.count = 0
        self._saved = {}

    def __enter__(self):
        import sys
        for n in self.NAMES:
            orig = getattr(torch.Tensor, n)
            self._saved[n] = orig

            def wrap(t, *a, _orig=orig, **k):
                f = sys._getframe(1)
                if f.f_code.co_name == "train_mode" and f.f_code.co_filename.endswith("train.py"):
                    self.count += 1
                return _orig(t, *a, **k)
            setattr(torch.Tensor, n, wrap)
        return self

    def __exit__(self, *exc):
        for n, orig in self._saved.items():
            setattr(torch.Tensor, n, orig)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    with HostReads() as reads:
        params, losses = tr.train_mode(_args(), small_plan(), torch.device("cpu"), rank=rank,
                                       world=world, stepper_cls=OracleStepper, log=lambda s: None)
    q.put((rank, params, losses, reads.count))
    dist.destroy_process_group()


def test_shard_schedule():
    steps, idx = tr.shard_schedule(10, 4, 1, 2)
    assert steps == 2 and idx.tolist() == [2, 3, 6, 7]
    steps, idx = tr.shard_schedule(8, 4, 0, 1)
    assert idx.tolist() == list(range(8))
    with pytest.raises(ValueError):
        tr.shard_schedule(8, 3, 0, 2)             # not a multiple of the ranks
    with pytest.raises(ValueError):
        tr.shard_schedule(3, 4, 0, 1)             # less than one global batch


def test_two_rank_gloo_train_mode_matches_one_rank():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    got = {r: (p, l) for r, p, l, _ in res}
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # the loop reads the per-step losses once per epoch, not once per step
    assert all(n == _args().num_epochs for *_, n in res), [n for *_, n in res]
    one, one_losses = tr.train_mode(_args(), small_plan(), torch.device("cpu"),
                                    stepper_cls=OracleStepper, log=lambda s: None)
    np.testing.assert_array_equal(got[0][0], got[1][0])          # identical replicas
    assert len(got[0][1]) == len(one_losses) == 4                 # 2 epochs x 2 steps
    np.testing.assert_allclose(got[0][0], one, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(got[0][1], one_losses, rtol=1e-12)
    # the parameters moved
    p0 = fs.init_params(small_plan().Nmax, seed=0).numpy()
    start = np.concatenate([p0[k].astype(np.float64).reshape(-1) for k in GRAD_ORDER])
    assert np.abs(one - start).max() > 1e-4
