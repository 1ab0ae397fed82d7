"""bench.py's timed region replays the steps from a HIP graph, batches
alternating over two streams forked from and joined back to the capture
stream (bench.GraphSteps).  The replay must compute what eager launches of
the same plans compute: pred / h / metrics bit for bit (same kernels, same
inputs), every batch's outputs written, and the join must order the side
stream's work before the capture stream's next use."""
import pytest
import torch

import bench
from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd.synthetic import make_batch

pytestmark = pytest.mark.gpu


def _plans(gpu, streams, K=4, S=64, Nmax=32, H=128):
    params = fs.init_params(Nmax, seed=0, device=gpu)
    plans = []
    for k in range(K):
        t = make_batch(S, Nmax, H, seed=40 + k).to_device(gpu)
        out = fs.StepOutputs(pred=torch.zeros(fs.pred_shape(S, 20, Nmax, "ped"), device=gpu),
                             h=torch.full((S, 16, H), float("nan"), device=gpu),
                             metrics=torch.full((S, 8), float("nan"), device=gpu))
        plans.append(fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                                 t["h0"], n_frames=t["n_frames"], ped_mask=t["ped_mask"], out=out,
                                 stream=streams[k % len(streams)], pred_layout="ped"))
    return plans


@pytest.mark.parametrize("nstreams", [1, 2])
def test_graph_replay_matches_eager(gpu, nstreams):
    streams = [torch.cuda.Stream(device=gpu) for _ in range(nstreams)]
    plans = _plans(gpu, streams)
    K = len(plans)
    for p in plans:
        p.run()
    torch.cuda.synchronize()
    eager = [(p.out.pred.clone(), p.out.h.clone(), p.out.metrics.clone()) for p in plans]
    assert all(torch.isfinite(e[1]).all() for e in eager)
    for p in plans:                              # poison: the replay must write every output
        p.out.h.fill_(float("nan"))
        p.out.metrics.fill_(float("nan"))
    torch.cuda.synchronize()
    g = bench.GraphSteps(lambda i: plans[i % K].run(), K, streams[0], side=streams[1:])
    g.replay()
    torch.cuda.synchronize()
    for p, (pred, h, m) in zip(plans, eager):
        assert torch.equal(p.out.pred, pred)
        assert torch.equal(p.out.h, h)
        assert torch.equal(p.out.metrics, m)
    # the join: a read on the capture stream after the replay sees the side
    # stream's batches complete
    g.replay()
    probe = torch.stack([p.out.h.sum() for p in plans[1::2]]) if nstreams == 2 else None
    torch.cuda.synchronize()
    if probe is not None:
        assert torch.equal(probe.cpu(), torch.stack([e[1].sum() for e in eager[1::2]]).cpu())


def test_graph_event_time_positive(gpu):
    streams = [torch.cuda.Stream(device=gpu)]
    plans = _plans(gpu, streams, K=2)
    g = bench.GraphSteps(lambda i: plans[i % 2].run(), 8, streams[0])
    dt = bench.graph_event_time(g, streams[0])
    # one 64-scene launch: microseconds, not the replay's host call alone
    assert 1e-6 < dt < 1e-3
