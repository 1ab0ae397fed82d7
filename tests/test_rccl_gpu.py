"""GPU: the multi-rank train step's structure on RCCL,
rehearsed on one GPU with a one-rank nccl group: TrainStep(collective=True)
runs gradient -> RCCL all-reduce -> g2k_update_f32 on the plans' stream, and
the same steps captured in a HIP graph (the collective included) and
replayed.  Both must leave parameters, mean squares and the gradient buffer
bit-identical to the one-rank fused call (g2k_train_step_f32 with the
update: the same row sum and update arithmetic in one launch fewer); a
one-rank all-reduce is the identity.  Then bench.py --collective on runs the
structure end to end, captured (its default) and from host launches
(--eager-collective).  Every capture that holds a collective follows
dist.reap_pending_work: synchronize, then ProcessGroup._wait_for_pending_works
until the watchdog holds no eager Work — the watchdog's hipEventQuery of an
eager Work's end event, recorded on the RCCL stream the capture has put into
capture mode, was the r7m abort (hipErrorCapturedEvent).
test_capture_right_after_eager_collectives captures immediately after eager
collectives, several times over, with no pause.  The N > 1 data path is covered by the gloo
tests (tests/test_dist.py, tests/test_train_mode*.py); RCCL across GPUs is
measured by the driver's multi-GPU bench."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(port, q):
    import torch.distributed as dist

    from multimodaltraj_2_amd import frame_step as fs
    from multimodaltraj_2_amd.dist import reap_pending_work
    from multimodaltraj_2_amd.synthetic import make_batch
    from multimodaltraj_2_amd.train_step import TrainStep
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0", TORCH_NCCL_CUDA_EVENT_CACHE="0")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    try:
        b = make_batch(6, 32, 128, F=12, seed=3, h0_scale=1.0)
        t = b.to_device(dev)
        params = fs.init_params(32, seed=0, device=dev)
        s = torch.cuda.Stream(device=dev)

        def make(coll):
            return TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                             t["h0"], stride=b.stride, stream=s, collective=coll)

        fused, eager, graphed = make(False), make(True), make(True)
        assert not fused.collective and eager.collective
        steps = 4
        for _ in range(steps):
            gf = fused.run()
            ge = eager.run()
        graphed.run()                                 # eager: communicator + RCCL buffers
        reap_pending_work()                           # no eager Work left for the watchdog
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            for _ in range(steps - 1):
                gg = graphed.run()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        res = {k: (ts.flat.cpu().numpy(), ts.ms.cpu().numpy(), gr.cpu().numpy())
               for k, ts, gr in (("fused", fused, gf), ("eager", eager, ge), ("graph", graphed, gg))}
        # a second replay = more steps, the same as eager steps
        g.replay()
        for _ in range(steps - 1):
            eager.run()
        torch.cuda.synchronize()
        res["replay2"] = (graphed.flat.cpu().numpy(), eager.flat.cpu().numpy())
        q.put(res)
    finally:
        dist.destroy_process_group()


def test_one_rank_rccl_step_structure_bit_identical(gpu):
    import torch.multiprocessing as mp

    from tests.test_train_mode import _port
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    f, e, gr = res["fused"], res["eager"], res["graph"]
    for a, b_ in ((f, e), (f, gr)):
        for x, y in zip(a, b_):
            np.testing.assert_array_equal(x, y)
    assert np.any(f[0] != 0) and f[2][-1] > 0         # stepped, count > 0
    np.testing.assert_array_equal(*res["replay2"])


def _cycles_worker(port, cycles, q):
    """Eager collectives (all-reduce, barrier) and, with no pause, a capture
    holding a collective — ``cycles`` times; then every graph replayed."""
    import torch.distributed as dist

    from multimodaltraj_2_amd.dist import reap_pending_work
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      HSA_ENABLE_IPC_MODE_LEGACY="0", TORCH_NCCL_CUDA_EVENT_CACHE="0")
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    try:
        s = torch.cuda.Stream(device=dev)
        buf = torch.ones(1283, device=dev)
        graphs = []
        for c in range(cycles):
            with torch.cuda.stream(s):
                for _ in range(3):                    # eager Works the watchdog lists
                    dist.all_reduce(buf)
                    buf.mul_(0.5)
            dist.barrier()
            reap_pending_work()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
                dist.all_reduce(buf)
                buf.add_(1.0)
            graphs.append(g)
        for g in graphs:
            g.replay()
        torch.cuda.synchronize()
        q.put(float(buf[0].item()))
    finally:
        dist.destroy_process_group()


def test_capture_right_after_eager_collectives(gpu):
    """The r7m race, provoked: eager collectives immediately before each of
    several captures (no sleep).  reap_pending_work makes it deterministic;
    the value checks every replayed all-reduce ran (one rank: identity)."""
    import torch.multiprocessing as mp

    from tests.test_train_mode import _port
    cycles = 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_cycles_worker, args=(_port(), cycles, q))
    p.start()
    v = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    want = 1.0
    for _ in range(cycles):                           # eager: 3 halvings, capture: + 1 (not run)
        want *= 0.125
    want += cycles                                    # the replays: + 1 each
    assert v == want


@pytest.mark.parametrize("capture", [False, True], ids=["host_launches", "captured"])
def test_bench_collective_structure(gpu, capture):
    """bench.py --collective on: the train line reports the gradient ->
    all-reduce -> update structure and its parts' times; one HIP graph with
    the collective captured by default, host launches with --eager-collective."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--collective", "on", "--steps", "10",
           "--warmup", "3", "--no-cpu-baseline", "--config", "eth_hotel_synth", "--rotate", "4"]
    if not capture:
        cmd.append("--eager-collective")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    tm = line["train_mode"]
    assert tm["step_structure"].startswith("gradient -> RCCL all-reduce -> update")
    assert ("captured" in tm["step_structure"]) == capture
    parts = tm["collective_parts_us"]
    assert set(parts) == {"gradient", "allreduce", "update"} and all(v > 0 for v in parts.values())
    print(json.dumps({"capture": capture, "ms_per_step": tm["ms_per_step"], "parts_us": parts}))
