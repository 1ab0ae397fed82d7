#!/usr/bin/env python3
"""bench.py — frames/sec of the g2k_lstm_mcr per-frame train step on MI355X.

One step = one pass of the fused per-frame body (train.py:197-276: window
norms, embeddings, g2k_lstm_mcr forward, attention + hidden recurrence,
ADE/FDE sums) over one batch of synthetic ETH-shaped scenes, inputs resident
in HBM.  This is "reference mode": the reference's train.py loop has no loss
or backward (SURVEY.md finding 5).  The build's train mode (the same step +
loss gradient + one gradient all-reduce + RMSProp) is timed beside it under
"train_mode", with its own roofline.
Workload = BASELINE.json configs[1]: "eth_hotel_synth" (S=256 scenes per
rank, Nmax=32 peds, H=128, F=20 frames).  Weak scaling: every rank owns its
own 256 scenes (seeded per rank); reference mode has no data-path collective
(the ADE/FDE numerators are summed across ranks once after the timed loop).

Inputs rotate over K device-resident batches whose total exceeds the 256 MiB
Infinity Cache (``--rotate``), so the HBM figure is not served on-die.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]

With N > 1 and no WORLD_SIZE in the environment this process launches N
ranks itself (``python -m torch.distributed.run``, one rank per GPU, RCCL)
before it touches the GPU, and relays the ranks' output; a worker whose
process group is not N ranks wide fails.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multimodaltraj_2_amd import frame_step as fs          # noqa: E402
from multimodaltraj_2_amd.dist import reap_pending_work     # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, FRAMES_PER_SCENE, make_batch  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MALL_BYTES = 256 * 2 ** 20     # Infinity Cache: rotate past this many bytes
METRIC = "frames/sec (obs=8,pred=12) g2k_lstm_mcr train step; ADE/FDE vs reference"
REAL = "eth_ucy_real"          # config 3's workload on real data (multimodaltraj_2_amd/realdata.py)


# ---------------------------------------------------------------------------
# algorithmic bytes: compulsory HBM traffic of one launch
# ---------------------------------------------------------------------------
def algorithmic_bytes(b, H, params_bytes, targets_shared=False):
    """One g2k_step_fused_f32 launch: reads the ACTIVE pedestrians' positions
    (W rows), vislet and targets (F frames x 24 floats; one frame's with
    shared targets), G, h_in, n_active and the weights; writes pred for the
    active pedestrians, h_out and the metrics row."""
    S, W, Nmax, _ = b.pos.shape
    L2, D, T = 24, 16, 8
    F = b.n_frames.astype(np.int64) if b.n_frames is not None else b.F
    FT = np.minimum(F, 1) if targets_shared else F
    nact = b.n_active.astype(np.int64)
    extra = S * 4 + S * Nmax if b.n_frames is not None else 0      # n_frames, ped_mask
    rd = (W * nact * 8).sum() + (2 * nact * 4).sum() + S * D * T * 4 \
        + (FT * nact * L2 * 4).sum() + S * D * H * 4 + S * 4 + params_bytes + extra
    wr = (F * L2 * nact * 4).sum() + S * D * H * 4 + S * 8 * 4
    return int(rd + wr)


# ---------------------------------------------------------------------------
# algorithmic flops: the roof a launch is bound by
# ---------------------------------------------------------------------------
FP32_PEAK_TFS = 157.3          # MI355X_MICROARCH.md: FP32 vector = FP32 MFMA (16x16x4 f32) peak
RIDGE = FP32_PEAK_TFS * 1e12 / (HBM_PEAK_GBS * 1e9)      # 19.7 flop/B
GRID_LSTM_FLOPS = 16 * (16 // 4) * 126                     # D * (D/4) * 126 = 8,064 per frame


def flops_per_frame(n, H, grid_lstm=False):
    """F_frame = 776 N + 20,000 + 672 H for one (scene,
    frame) unit of train.py:197-276 with N active pedestrians — embed 2TND +
    2D^2T, vislet 4ND, E 2T(D+2)D + TD, Rm 4TD, A 2D^2T + TD, Cst 2DT^2, Y
    48T^2 + 48TN, the attention softmax ~5D^2, the recurrence 2D^2H + 10DH,
    the errors ~72N (D 16, T 8; transcendentals one flop each; the constant
    terms sum to 19,968, which the survey rounds to 20,000 and so do we);
    + 8,064 with the GridLSTM encoder (helper.py:31-39)."""
    return 776 * n + 20_000 + 672 * H + (GRID_LSTM_FLOPS if grid_lstm else 0)


def bwd_flops_per_frame(n, loss="l2"):
    """The train mode's gradient of one frame (the loss's dependency cone:
    pred = (Wc (E g)) Wo with E = Wv X + bv, X = [Wii (Bv Wi); vislet Wi];
    A and the recurrence do not reach pred, train.py:254).  dY 72N (L2: the
    residual, its square and sum) or ~480N (the bivariate-Gaussian NLL and
    its gradient, 40 flops per (pedestrian, step)); dWo = M^T dY and dM = dY
    Wo^T 384N each; dWc = dM Cst^T and dCst = Wc^T dM 3,072 each; dE =
    dCst g^T 2,048; dWv = dE X^T and dX = Wv^T dE 4,608 each, dbv 128; dWii
    = dX0 U^T and dU = Wii^T dX0 4,096 each; dWi = Bv^T dU + vislet^T dVe
    256N + 64N (data, g and G get no gradient)."""
    return (72 if loss == "l2" else 480) * n + 384 * n * 2 + 256 * n + 64 * n + 25_728


def _frames_and_active(b):
    F = b.n_frames.astype(np.int64) if b.n_frames is not None else np.full(b.S, b.F, np.int64)
    return F, b.n_active.astype(np.int64)


def algorithmic_flops(b, H, grid_lstm=False):
    """Flops of one g2k_step_fused_f32 launch: every scene's frames at its
    active pedestrian count."""
    F, n = _frames_and_active(b)
    return int((F * flops_per_frame(n, H, grid_lstm)).sum())


def train_algorithmic_flops(b, H, P, loss="l2"):
    """One train step: the forward's flops, the gradient's, the fixed-order
    sum of the per-scene [P + 2] rows and the RMSProp + clip update (~8 per
    parameter)."""
    F, n = _frames_and_active(b)
    return algorithmic_flops(b, H) + int((F * bwd_flops_per_frame(n, loss)).sum()) \
        + b.S * (P + 2) + 8 * P


def roofline(abytes, aflops, kern_s, step_s):
    """The contract's roofline object for one kernel: ``bound`` by the
    launch's arithmetic intensity against the FP32 ridge (157.3 TF/s over 8
    TB/s = 19.7 flop/B): "hbm" (achieved in GB/s) or "mfma" (the FP32 compute
    roof — on gfx950 the f32 MFMA and the vector peak are the same 157.3
    TF/s; achieved in TFLOP/s).  Both fractions are carried for one launch
    (kern_s) and per step of the timed loop (step_s)."""
    inten = aflops / abytes
    f_hbm, f_fl = abytes / kern_s / 1e9 / HBM_PEAK_GBS, aflops / kern_s / 1e12 / FP32_PEAK_TFS
    p_hbm, p_fl = abytes / step_s / 1e9 / HBM_PEAK_GBS, aflops / step_s / 1e12 / FP32_PEAK_TFS
    compute = inten >= RIDGE
    r = {"bound": "mfma" if compute else "hbm",
         "achieved": aflops / kern_s / 1e12 if compute else abytes / kern_s / 1e9,
         "peak": FP32_PEAK_TFS if compute else HBM_PEAK_GBS,
         "unit": "TFLOP/s" if compute else "GB/s"}
    r["frac"] = r["achieved"] / r["peak"]
    r.update({"algorithmic_bytes": int(abytes), "flops": int(aflops), "intensity": inten,
              "ridge": RIDGE, "frac_hbm": f_hbm, "frac_flops": f_fl,
              "frac_hbm_per_step": p_hbm, "frac_flops_per_step": p_fl,
              "achieved_per_step": (aflops / step_s / 1e12) if compute else abytes / step_s / 1e9,
              "bound_note": "mfma = the FP32 compute roof (f32 MFMA = vector peak, 157.3 TF/s)"
                            if compute else "HBM roof (8 TB/s)"})
    return r


def train_algorithmic_bytes(b, H, params_bytes, P, targets_shared=False):
    """One train step (forward outputs + gradient + update): the forward's
    bytes, the [P + 2] gradient written and read back, the parameters and the
    RMSProp mean squares read and written once."""
    return algorithmic_bytes(b, H, params_bytes, targets_shared) + 2 * (P + 2) * 4 + 4 * P * 4


# ---------------------------------------------------------------------------
# CPU baseline: the float64 oracle in the reference's loop
# structure, on the GPU box's host cores, before the GPU is touched
# ---------------------------------------------------------------------------
def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _oracle_scenes(b, params_np, lo, hi, budget_s, threads):
    """Scenes lo, lo+1, ... < hi through oracle.scene_step (one scene at a
    time, the reference's per-batch loop) until budget_s has elapsed;
    returns (frames, seconds)."""
    from threadpoolctl import threadpool_limits
    from oracle import g2k_ref as ref
    frames = 0
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        s = lo
        while True:
            nf = int(b.n_frames[s]) if b.n_frames is not None else b.F
            pm = b.ped_mask[s].astype(bool) if b.ped_mask is not None else None
            ref.scene_step(b.pos[s], b.vislet[s], b.G[s], params_np, b.targets[s],
                           b.n_active[s], b.h0[s], n_frames=nf, stride=b.stride, ped_mask=pm)
            frames += nf
            s = s + 1 if s + 1 < hi else lo
            if time.perf_counter() - t0 > budget_s:
                break
        return frames, time.perf_counter() - t0


def job_cpus():
    """CPUs this job may use: the affinity mask, capped by a cgroup CPU quota
    and by the job's declared CPU share (OMP_NUM_THREADS: the GPU box sets it
    to the job's share of its host, 16 of 256 threads per GPU)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        n = min(n, int(share))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def _pool_worker(a):
    b, p, lo, hi, budget = a
    return _oracle_scenes(b, p, lo, hi, budget, 1)


def cpu_baseline(cfg, b, params_np, budget_s, procs):
    """Three denominators: one process with one BLAS thread
    (how the reference runs: one Python process, tiny matrices), one process
    with all BLAS threads, and the all-core aggregate (``procs`` processes on
    disjoint scenes, spawned before this process touches the GPU)."""
    import multiprocessing as mp
    S = b.S
    f1, t1 = _oracle_scenes(b, params_np, 0, S, budget_s, 1)
    fa, ta = _oracle_scenes(b, params_np, 0, S, budget_s / 2, None)
    per = max(1, S // procs)
    jobs = [(b, params_np, (i * per) % S, min(S, (i * per) % S + per), budget_s / 2)
            for i in range(procs)]
    ctx = mp.get_context("spawn")
    pool = ctx.Pool(procs)
    try:
        res = pool.map(_pool_worker, jobs)
    finally:
        pool.close()          # let the workers exit on their own (no SIGTERM on teardown)
        pool.join()
    agg = sum(f for f, _ in res) / max(t for _, t in res)
    return {"value": f1 / t1, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"the float64 NumPy oracle (oracle/g2k_ref.py) in train.py's per-scene loop, "
                      f"{f1} frames of the same workload's scenes in {t1:.1f} s, "
                      f"1 thread (the reference's TF path cannot run here: no TF 1.x)",
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "job_cpus": job_cpus(),
            "blas_all_threads": {"value": fa / ta, "unit": "frames/s", "seconds": round(ta, 2)},
            "all_core_aggregate": {"value": agg, "unit": "frames/s", "processes": procs,
                                   "note": "disjoint scene slices, one BLAS thread each, one "
                                           "process per CPU this job may use (job_cpus; the "
                                           "host's other threads belong to other jobs)"}}


# ---------------------------------------------------------------------------
# multi-rank launcher (the parent never initialises the GPU)
# ---------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------
# timing
# ---------------------------------------------------------------------------
def timed(step, n, warmup, dist, sync):
    """W untimed steps, then K steps bracketed by barrier + synchronize on
    both sides; returns the max over ranks of the elapsed seconds."""
    for i in range(warmup):
        step(i)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(n):
        step(i)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([el], dtype=torch.float64,
                         device="cuda" if torch.cuda.is_initialized() else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    return el


def event_time(step, reps, stream):
    """Average seconds per step from HIP events recorded on the stream the
    kernels are launched on."""
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for i in range(reps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / 1e3 / reps


_HIP = None


def upload_graph(g, stream):
    """hipGraphUpload of a captured graph's executable on ``stream`` (its
    one-time device-side setup, done at capture time instead of inside the
    first timed replay; runs no step).  G2K_BENCH_NO_UPLOAD=1 skips it (A/B)."""
    global _HIP
    if os.environ.get("G2K_BENCH_NO_UPLOAD"):
        return
    import ctypes
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipGraphUpload.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        _HIP.hipGraphUpload.restype = ctypes.c_int
    rc = _HIP.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()), ctypes.c_void_p(stream.cuda_stream))
    if rc != 0:
        raise RuntimeError(f"hipGraphUpload failed: {rc}")
    torch.cuda.synchronize()


class GraphSteps:
    """Steps replayed from a HIP graph (torch.cuda.CUDAGraph over the plans'
    stream): ``n`` consecutive calls of ``step(i0 + i)`` captured once, then
    one graph launch runs all of them back to back on the GPU — the host's
    per-launch cost (Python, the C ABI's checks, hipLaunchKernel) no longer
    paces a ~20 us step.  ``run(i)`` with i a multiple of ``n`` replays it."""

    def __init__(self, step, n, stream, i0=0, side=(), thread_local=False):
        self.n = n
        self.g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        if thread_local:
            # a process group is up: no eager Work may be left for its
            # watchdog to query while the capture holds the RCCL stream
            # (multimodaltraj_2_amd/dist.py reap_pending_work)
            reap_pending_work()
        # thread_local: a capture that holds an RCCL collective (the process
        # group's watchdog thread keeps querying its events meanwhile)
        with torch.cuda.graph(self.g, stream=stream,
                              capture_error_mode="thread_local" if thread_local else "global"):
            for s in side:                     # forked from the capture stream ...
                s.wait_stream(stream)
            for i in range(n):
                step(i0 + i)
            for s in side:                     # ... and joined back
                stream.wait_stream(s)
        torch.cuda.synchronize()
        upload_graph(self.g, stream)

    def replay(self):
        self.g.replay()


def timed_graph(step, n, warmup, dist, sync, stream, side=(), thread_local=False):
    """timed() with the warm-up and the timed steps each as one graph replay
    (exactly ``n`` steps between the barriers)."""
    gw = GraphSteps(step, max(warmup, 1), stream, side=side, thread_local=thread_local)
    gm = GraphSteps(step, n, stream, i0=max(warmup, 1), side=side, thread_local=thread_local)
    gw.replay()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    gm.replay()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    el = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    return el, gm


def collective_parts(ts, stream, K, graph, reps=50):
    """The multi-rank step's parts timed alone with HIP events on the plans'
    stream (µs each; replayed from a HIP graph of ``reps`` copies when
    ``graph``, else host launches): gradient (scene kernel + row sum), the
    all-reduce of the [P + 2] buffer, the update (DESIGN.md §8's budget)."""
    from multimodaltraj_2_amd.dist import allreduce_grad
    from multimodaltraj_2_amd.train_step import optimizer_update
    g = ts.run(0)
    kw = dict(lr=ts.lr, decay=ts.decay, grad_clip=ts.grad_clip)
    fns = {"gradient": lambda i: ts._slots[i % K].run(),
           "allreduce": lambda i: allreduce_grad(g, ts.group, force=True),
           "update": lambda i: optimizer_update(ts.flat, g, ms=ts.ms, stream=stream, **kw)}
    parts = {}
    with torch.cuda.stream(stream):
        for k, fn in fns.items():
            if graph:
                parts[k] = graph_event_time(GraphSteps(fn, reps, stream, thread_local=True), stream)
            else:
                parts[k] = event_time(fn, reps, stream)
    return {k: v * 1e6 for k, v in parts.items()}


def graph_event_time(g, stream):
    """Average seconds per step of a captured graph's replay, from HIP events
    on the stream the replay is launched on (the current stream: the graph's
    kernels run there, not on the capture stream)."""
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    cur = torch.cuda.current_stream()
    g.replay()
    ev0.record(cur)
    g.replay()
    ev1.record(cur)
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / 1e3 / g.n


def load_pmc(name):
    """(HBM bytes per launch, provenance) from the committed PMC profile
    profiles/pmc_<name>.json — a STATIC value, collected by tools/gpu_round.sh
    in separate rocprofv3 --pmc passes (FETCH_SIZE x2 + WRITE_SIZE), not in this
    run; ``matches_current_tree`` says whether it was taken on the kernel
    sources this run built from (build.kernel_tree_sha)."""
    from multimodaltraj_2_amd.build import kernel_tree_sha
    rel = os.path.join("profiles", f"pmc_{name}.json")
    p = os.path.join(ROOT, rel)
    if not os.path.exists(p):
        return None, None
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    sha = d.get("kernel_tree_sha")
    return d.get("hbm_bytes_per_launch"), {
        "file": rel, "kind": "static profile (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                            "of bench.py, tools/gpu_round.sh), not measured in this run",
        "kernel_tree_sha": sha, "matches_current_tree": sha == kernel_tree_sha()}


def real_scene_batch(S, H, rank, world):
    """Config 3's workload on real data: the k-fold-4 training datasets plus
    ETH hotel (multimodaltraj_2_amd/realdata.py: distinct sample.py scenes,
    natively planned), S per rank, rank r taking the r-th contiguous shard of
    the S * world global scenes.  Data: the reference's CSV arrays committed
    under tests/golden/ (the bench's input files; the product reads a data
    root)."""
    from multimodaltraj_2_amd import realdata as rd
    from multimodaltraj_2_amd.synthetic import SceneBatch
    from multimodaltraj_2_amd.train import plan_subset
    raw = {n: np.load(os.path.join(ROOT, "tests", "golden", f"data_{n}.npz"))["raw_data"]
           for n in rd.fold_datasets(4)}
    plan = rd.plan_scenes(S * world, raw)
    sub = plan_subset(plan, np.arange(rank * S, (rank + 1) * S))
    h = sub.host()
    rng = np.random.default_rng(1 + rank)
    return SceneBatch(pos=h["pos"], vislet=h["vislet"],
                      G=rng.standard_normal((S, 16, 8)).astype(np.float32), targets=h["targets"],
                      n_active=h["n_active"], h0=np.zeros((S, 16, H), np.float32), stride=0,
                      n_frames=h["n_frames"], ped_mask=h["ped_mask"])


def selftest_worker(args, world, rank):
    """--selftest-launcher (CPU, gloo): the launcher, the process-group check,
    the timing brackets and the metric all-reduce, with a no-op step in place
    of the HIP kernel (tests/test_bench_launcher.py)."""
    import torch.distributed as dist
    dist.init_process_group("gloo")
    if dist.get_world_size() != args.gpus:
        raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    world = dist.get_world_size()
    metrics = torch.full((4, 8), float(rank + 1), dtype=torch.float64)
    el = timed(lambda i: None, args.steps, args.warmup, dist, lambda: None)
    tot = metrics.sum(dim=0)
    dist.all_reduce(tot)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "selftest": True, "elapsed_s": el,
                          "metric_sums": tot.tolist()}), flush=True)
    dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="eth_hotel_synth", choices=sorted(CONFIGS) + [REAL])
    ap.add_argument("--scenes", type=int, default=0, help="override scenes per rank")
    ap.add_argument("--rotate", type=int, default=0,
                    help="input batches to rotate over (0: enough to exceed the 256 MiB MALL)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="processes of the all-core CPU aggregate (0: the CPUs this job may use)")
    ap.add_argument("--no-train", action="store_true", help="skip the train-mode timing")
    ap.add_argument("--loss", choices=("l2", "nll"), default="l2",
                    help="train-mode loss: 1/2 squared error or the bivariate-Gaussian NLL")
    ap.add_argument("--pred-layout", choices=("ped", "band"), default="ped",
                    help="pred as [S, F, Nmax, L, 2] (the per-pedestrian view train.py:254 "
                         "transposes to; only active pedestrians written) or pred_path_band "
                         "[S, F, 2L, Nmax]")
    ap.add_argument("--split", type=int, default=0,
                    help="workgroups per scene (G2K_STEP_SPLIT; 0: automatic, enough to cover "
                         "the CUs when a rank has fewer scenes than CUs)")
    ap.add_argument("--streams", type=int, default=16,
                    help="reference mode: consecutive (independent) batches on this many "
                         "streams in turn, so launches overlap (the roofline still divides by "
                         "one launch's duration).  16: the timed steps' launches are all queued "
                         "at once, so a CU's freed workgroup slot is refilled from the next "
                         "launch at once (profiles/r11m_streams_sweep.txt: eth_hotel_synth "
                         "14.3 -> 13.7-13.9 us per step at 20 steps against 4 streams, 12.5 -> "
                         "11.8 at 200; every config gains)")
    ap.add_argument("--coresident", choices=("auto", "on", "off"), default="auto",
                    help="reference mode: G2K_STEP_CORESIDENT (two 8-wave workgroups per CU "
                         "while launches are in flight); auto = on with 2 or more streams")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step from the host instead of replaying the timed steps "
                         "from a HIP graph")
    ap.add_argument("--collective", choices=("auto", "on"), default="auto",
                    help="train mode: the multi-rank step structure (gradient -> RCCL all-reduce "
                         "-> update); auto = when WORLD_SIZE > 1, on = also on one rank (a "
                         "one-rank nccl group: the structure measured on one GPU)")
    ap.add_argument("--eager-collective", action="store_true",
                    help="train mode, collective structure: launch gradient -> RCCL all-reduce "
                         "-> update from the host every step instead of replaying the steps, "
                         "collective included, from one HIP graph (the default)")
    ap.add_argument("--selftest-launcher", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args(argv)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.selftest_launcher:
        return selftest_worker(args, world, rank)

    if args.config == REAL:
        b = real_scene_batch(args.scenes or 128, 128, rank, world)
        S, H, Nmax, F = b.S, 128, b.pos.shape[2], b.F
    else:
        cfg = dict(CONFIGS[args.config])
        if args.config in ("eth_ucy_loo_kfold4", "dense_crowd"):
            cfg["S"] = cfg["S"] // 8          # 128 scenes per GPU
        S = args.scenes or cfg["S"]
        Nmax, H, F = cfg["Nmax"], cfg["H"], FRAMES_PER_SCENE
        b = make_batch(S, Nmax, H, F=F, seed=1 + rank)
    params_host = fs.init_params(Nmax, seed=0)

    # CPU baseline first: its worker processes are spawned before this
    # process initialises the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        procs = args.cpu_procs or job_cpus()
        cpu = cpu_baseline(args.config, b, params_host.numpy(), args.cpu_budget, procs)

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1 or args.collective == "on":
        import torch.distributed as dist
        if not args.eager_collective:
            # no ProcessGroupNCCL event recycled from a captured Work (its last
            # record inside a capture) into an eager Work the watchdog polls
            # (the race itself is closed by reap_pending_work)
            os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
        if world == 1:                   # a one-rank group (--collective on)
            for k, v in dict(MASTER_ADDR="127.0.0.1", RANK="0", WORLD_SIZE="1").items():
                os.environ.setdefault(k, v)
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("nccl", device_id=dev)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    params = params_host.to(dev)
    pbytes = sum(getattr(params, k).numel() * 4 for k in ("Wi", "Wii", "Wv", "bv", "Wr", "Wc", "Wo"))
    shared = args.config == REAL          # real scenes: one target set per scene (every frame's)
    stream = torch.cuda.Stream(device=dev)   # the plans' stream (graph capture needs a non-default one)
    layout = dict(pred_layout=args.pred_layout, targets_shared=shared, frames=F if shared else None,
                  split=args.split)
    cores = args.coresident == "on" or (args.coresident == "auto" and args.streams >= 2)
    abytes = algorithmic_bytes(b, H, pbytes, shared)
    K = args.rotate or max(1, -(-MALL_BYTES // abytes) + 1)
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(max(args.streams, 1) - 1)]
    K = -(-K // len(streams)) * len(streams)     # batch k always on stream k % streams

    # K device-resident input batches (the base batch plus small per-batch
    # position offsets, so no two share a cache line) and their plans
    base = b.to_device(dev)
    if shared:
        base["targets"] = base["targets"][:, :1].contiguous()
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    batches, plans = [], []
    for k in range(K):
        t = {key: (v.clone() if isinstance(v, torch.Tensor) else v) for key, v in base.items()}
        if k:
            t["pos"].add_(1e-3 * torch.randn(t["pos"].shape, device=dev, generator=gen))
            t["targets"].add_(1e-3 * torch.randn(t["targets"].shape, device=dev, generator=gen))
        out = fs.StepOutputs(pred=torch.zeros(fs.pred_shape(S, F, Nmax, args.pred_layout), device=dev),
                             h=torch.empty((S, 16, H), device=dev),
                             metrics=torch.empty((S, 8), device=dev))
        batches.append(t)
        plans.append(fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"],
                                 t["n_active"], t["h0"], n_frames=t["n_frames"],
                                 ped_mask=t["ped_mask"], stride=b.stride, out=out,
                                 stream=streams[k % len(streams)], coresident=cores, **layout))

    def step(i):
        plans[i % K].run()

    if args.no_graph:
        elapsed = timed(step, args.steps, args.warmup, dist, torch.cuda.synchronize)
    else:
        # (a process group is up: its watchdog thread queries events while we
        # capture, so the capture is thread-local)
        elapsed, gm = timed_graph(step, args.steps, args.warmup, dist, torch.cuda.synchronize, stream,
                                  side=streams[1:], thread_local=dist is not None)
    # reference mode: replicas only; the ADE/FDE numerators of the last batch
    # are summed across ranks once at the end
    tot = plans[(args.steps - 1) % K].out.metrics.double().sum(dim=0)
    if dist is not None:
        dist.all_reduce(tot)
    # the roofline's time: ONE launch's duration, launches back to back on
    # one stream (no overlap; what rocprofv3 reports per dispatch), over the
    # batches of stream 0
    R = max(20, min(args.steps, 200))
    one = [plans[k] for k in range(0, K, len(streams))]
    if args.no_graph:
        kern_s = event_time(lambda i: one[i % len(one)].run(), R, stream)
    else:
        kern_s = graph_event_time(GraphSteps(lambda i: one[i % len(one)].run(), R, stream,
                                             thread_local=dist is not None), stream)
    aflops = algorithmic_flops(b, H)

    train = None
    if not args.no_train:
        train = time_train(args, params, batches, dev, dist, S, F, H, world, b, pbytes, K, layout,
                           stream)

    if rank == 0:
        pmc = load_pmc(args.config)
        m = tot.cpu().numpy()
        line = {
            "metric": METRIC,
            "value": b.frames * world * args.steps / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("real (distinct sample.py scenes of the reference's ETH/UCY files, k-fold-4 "
                     "training datasets + ETH hotel; stride 0, n_frames = len(batch); N(0,1) "
                     "weights)" if args.config == REAL else
                     "synthetic (seeded random-walk ETH-shaped scenes; N(0,1) weights)"),
            "mode": "reference (train.py:197-276: forward, recurrence, ADE/FDE; the reference "
                    "has no backward)",
            "config": {"workload": args.config, "scenes_per_gpu": S, "global_scenes": S * world,
                       "frames_per_scene": F if b.n_frames is None else float(b.n_frames.mean()),
                       "frames_per_step": b.frames, "obs_len": 8, "pred_len": 12, "Nmax": Nmax,
                       "hidden": H, "D": 16, "parallelism": f"dp{world}",
                       "input_batches_rotated": K, "pred_layout": args.pred_layout,
                       "targets_shared": shared,
                       "workgroups_per_scene": fs.step_split(S, F, H, Nmax, b.pos.shape[1], b.stride,
                                                             args.split, cores,
                                                             targets_shared=shared),
                       "coresident": cores,
                       "workgroups_per_cu": fs.step_coresidency(S, F, H, Nmax, b.pos.shape[1], b.stride,
                                                                cores, shared),
                       "streams": len(streams),
                       "launch": "host launch per step" if args.no_graph else
                                 "HIP graph of the timed steps (one replay)"},
            # achieved: one launch alone (kern_s); *_per_step: the timed steps'
            # effective rate (launches overlap on streams / co-resident
            # workgroups, so it exceeds one launch's rate)
            "roofline": dict(roofline(abytes, aflops, kern_s, elapsed / args.steps),
                             traffic=pmc[0], traffic_source=pmc[1],
                             kernel="g2k_step_fused_f32 (g2k_scene_kernel)",
                             kernel_us=kern_s * 1e6),
            "cpu_baseline": cpu,
            "ade_fde_all_ranks": {"ADE": float(m[0] / max(m[1], 1)),
                                  "FDE_frob_per_frame": float(np.sqrt(m[2]) / max(m[5], 1))},
            "train_mode": train,
        }
        if cpu:
            v = line["value"]
            line["speedup_vs_cpu"] = {"one_thread": v / cpu["value"],
                                      "blas_all_threads": v / cpu["blas_all_threads"]["value"],
                                      "all_core_aggregate": v / cpu["all_core_aggregate"]["value"]}
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


def time_train(args, params, batches, dev, dist, S, F, H, world, b, pbytes, K, layout, stream):
    """--mode train: the same step plus loss gradient, ONE
    all-reduce of the flat [P + 2] gradient buffer across ranks (RCCL under
    the nccl backend) and the RMSProp update (multimodaltraj_2_amd/train_step.py).
    Timed like the reference-mode step over the same rotated batches."""
    from multimodaltraj_2_amd.train_step import TrainStep
    t0 = batches[0]
    if args.loss == "nll":
        params.head = torch.zeros((3, 12), device=dev)
    coll = world > 1 or args.collective == "on"
    ts = TrainStep(params, t0["pos"], t0["vislet"], t0["G"], t0["targets"], t0["n_active"],
                   t0["h0"], n_frames=t0["n_frames"], ped_mask=t0["ped_mask"], stride=b.stride,
                   loss=args.loss, stream=stream, collective=coll, **layout)
    for t in batches[1:]:
        ts.bind(t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"],
                n_frames=t["n_frames"], ped_mask=t["ped_mask"])
    last = {}

    def step(i):
        last["g"] = ts.run(i % K)

    # one rank: one C call per step (gradient + update); across ranks
    # gradient -> RCCL all-reduce -> update on the plans' stream.  Both are
    # replayed from a HIP graph, the collective captured beside the kernels
    # (one eager step first: the communicator and RCCL's own buffers exist
    # before capture; GraphSteps then reaps that step's Work from the
    # process group's watchdog before it captures); --eager-collective
    # launches the multi-rank steps from the host instead
    graph = not args.no_graph and not (coll and args.eager_collective)
    in_graph = False
    if graph and coll:
        step(0)
    if graph:
        el, gm = timed_graph(step, args.steps, args.warmup, dist, torch.cuda.synchronize, stream,
                             thread_local=dist is not None)
        kern_s = graph_event_time(gm, stream)
        in_graph = coll
    else:
        el = timed(step, args.steps, args.warmup, dist, torch.cuda.synchronize)
        kern_s = event_time(step, max(20, min(args.steps, 200)), stream)
    gl = last["g"].double().cpu().numpy()
    parts = collective_parts(ts, stream, K, graph) if coll else None
    abytes = train_algorithmic_bytes(b, H, pbytes, ts.P, layout["targets_shared"])
    aflops = train_algorithmic_flops(b, H, ts.P, args.loss)
    pmc = load_pmc(args.config + "_train")
    return {"metric": f"frames/sec (obs=8,pred=12) g2k_lstm_mcr train step + "
                      f"{'L2' if args.loss == 'l2' else 'bivariate-Gaussian NLL'} loss gradient + "
                      "gradient all-reduce + RMSProp update", "loss": args.loss,
            "value": b.frames * world * args.steps / el, "unit": "frames/s",
            "ms_per_step": el / args.steps * 1e3, "allreduce_bytes": int((ts.P + 2) * 4),
            "step_structure": ("gradient -> RCCL all-reduce -> update" + (
                " (HIP graph, collective captured)" if in_graph else " (host launches)"))
            if coll else "gradient + update in one call (one rank, HIP graph)"
            if graph else "gradient + update in one call (one rank, host launches)",
            "collective_parts_us": parts,
            "loss_per_prediction_last_step": float(gl[-2] / max(gl[-1], 1.0)),
            "optimizer": "RMSProp lr 0.005 decay 0.95, global-norm clip 10 (argParser.py:38-47)",
            # one step alone (the graph's steps back to back: kern_s) and the
            # timed loop's rate
            "roofline": dict(roofline(abytes, aflops, kern_s, el / args.steps),
                             traffic=pmc[0], traffic_source=pmc[1],
                             kernel=ts.kernel_names, step_us=kern_s * 1e6)}


if __name__ == "__main__":
    sys.exit(main())
