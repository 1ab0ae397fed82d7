"""GPU: the multi-rank train step's structure on RCCL,
rehearsed on one GPU with a one-rank nccl group: TrainStep(collective=True)
runs gradient -> RCCL all-reduce -> g2k_update_f32 on the plans' stream, and
the same steps captured in a HIP graph (the collective included) and
replayed.  Both must leave parameters, mean squares and the gradient buffer
bit-identical to the one-rank fused call (g2k_train_step_f32 with the
update: the same row sum and update arithmetic in one launch fewer); a
one-rank all-reduce is the identity.  Then bench.py --collective on runs the
structure end to end, from host launches (its default) and captured
(--capture-collective).  Captures run with TORCH_NCCL_CUDA_EVENT_CACHE=0 and
after a pause that lets the process group's watchdog reap the eager work
(without them its watchdog once queried a recycled event a capture held:
hipErrorCapturedEvent).  The N > 1 data path is covered by the gloo
tests (tests/test_dist.py, tests/test_train_mode*.py); RCCL across GPUs is
measured by the driver's multi-GPU bench."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(port, q):
    import torch.distributed as dist

    from multimodaltraj_2_amd import frame_step as fs
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
        torch.cuda.synchronize()
        time.sleep(0.5)                               # (bench.py time_train: watchdog reaps it)
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


@pytest.mark.parametrize("capture", [False, True], ids=["host_launches", "captured"])
def test_bench_collective_structure(gpu, capture):
    """bench.py --collective on: the train line reports the gradient ->
    all-reduce -> update structure and its parts' times; host launches by
    default, one HIP graph with --capture-collective."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--collective", "on", "--steps", "10",
           "--warmup", "3", "--no-cpu-baseline", "--config", "eth_hotel_synth", "--rotate", "4"]
    if capture:
        cmd.append("--capture-collective")
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
