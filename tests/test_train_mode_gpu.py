"""GPU: --mode train's HIP stepper (multimodaltraj_2_amd/train.py HipStepper:
the fold's real scenes gathered into HBM, one g2k_train_step_f32 plan per
step) against the float64 oracle stepper over the same steps: losses and the
parameters after k RMSProp steps, one rank (fused update) and the all-reduce
branch (gradient, then the separate update)."""
import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import train as tr
from tests.test_train_mode import OracleStepper, _args, small_plan

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [1, 2])
def test_hip_stepper_matches_oracle(gpu, world):
    args = _args()
    plan = small_plan()
    steps, idx = tr.shard_schedule(plan.S, args.train_batch, 0, 1)
    hip = tr.HipStepper(args, plan, idx, gpu, steps)
    ora = OracleStepper(args, plan, idx, torch.device("cpu"), steps)
    for e in range(args.num_epochs):
        for k in range(steps):
            if world == 1:
                g, r = hip.fused(k), ora.fused(k)
            else:                  # the all-reduce branch on one rank: grad, (sum), update
                g, r = hip.grad(k), ora.grad(k)
                hip.apply(g)
                ora.apply(r)
            g = g.double().cpu().numpy()
            r = r.numpy()
            assert abs(g[-2] - r[-2]) <= 1e-4 * r[-2] and g[-1] == r[-1]
            assert np.abs(g[:-2] - r[:-2]).max() <= 1e-4 * np.abs(r[:-2]).max()
    got, want = hip.params(), ora.params()
    assert np.abs(got - want).max() <= 1e-5 * max(1.0, np.abs(want).max())


def _gpu_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    params, losses = tr.train_mode(_args(), small_plan(), dev, rank=rank, world=world,
                                   log=lambda s: None)
    q.put((rank, params, losses))
    dist.destroy_process_group()


def test_two_rank_hip_train_mode_on_one_gpu(gpu):
    """The world > 1 branch end to end on the GPU: two ranks (gloo, both on
    cuda:0), each the HIP gradient of its shard, ONE all-reduce of the device
    [P + 2] buffer, g2k_update_f32 — identical replicas, equal to one rank
    over the union of the shards up to fp32 summation order."""
    import torch.multiprocessing as mp
    from tests.test_train_mode import _port
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (p, l)) for r, p, l in (q.get(timeout=240) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    one, one_losses = tr.train_mode(_args(), small_plan(), gpu, log=lambda s: None)
    np.testing.assert_array_equal(got[0][0], got[1][0])
    assert np.abs(got[0][0] - one).max() <= 1e-5 * max(1.0, np.abs(one).max())
    np.testing.assert_allclose(got[0][1], one_losses, rtol=1e-5)
