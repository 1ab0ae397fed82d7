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
