#!/usr/bin/env python3
"""bench.py — frames/sec of the g2k_lstm_mcr per-frame train step on MI355X.

One step = one pass of the fused per-frame body (train.py:197-276: window
norms, embeddings, g2k_lstm_mcr forward, attention + hidden recurrence,
ADE/FDE sums) over one batch of synthetic ETH-shaped scenes, inputs resident
in HBM.  Replicas only: the ADE/FDE numerators are summed across ranks once
after the timed loop.
Workload = BASELINE.json configs[1]: "eth_hotel_synth" (S=256 scenes per
rank, Nmax=32 peds, H=128, F=20 frames).  Weak scaling: every rank owns its
own 256 scenes (seeded per rank) — no data-path collective.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config NAME]
  (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N)

Prints ONE JSON line on rank 0 (see DESIGN.md §Measurement for the fields).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multimodaltraj_2_amd import frame_step as fs          # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, FRAMES_PER_SCENE, make_batch  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def algorithmic_bytes(b, H, params_bytes):
    """Compulsory bytes one launch of g2k_step_fused_f32 moves:
    reads pos/vislet/targets of ACTIVE pedestrians, G, h_in, n_active, weights;
    writes pred (all Nmax columns, padding zero-filled), h_out, metrics."""
    S, W, Nmax, _ = b.pos.shape
    F, L2, D, T = b.F, 24, 16, 8
    nact = b.n_active.astype(np.int64)
    rd = (W * nact * 8).sum() + (2 * nact * 4).sum() + S * D * T * 4 \
        + (F * nact * L2 * 4).sum() + S * D * H * 4 + S * 4 + params_bytes
    wr = S * F * L2 * Nmax * 4 + S * D * H * 4 + S * 8 * 4
    return int(rd + wr)


def cpu_baseline(b, params_np, budget_s=12.0):
    """The float64 oracle (oracle/g2k_ref.py) in the reference's loop
    structure, one scene at a time, one thread, on a bounded sample."""
    from threadpoolctl import threadpool_limits
    from oracle import g2k_ref as ref
    frames = 0
    scenes = 0
    with threadpool_limits(limits=1):
        t0 = time.perf_counter()
        while scenes < b.S:
            s = scenes
            ref.scene_step(b.pos[s], b.vislet[s], b.G[s], params_np, b.targets[s],
                           b.n_active[s], b.h0[s], n_frames=b.F, stride=b.stride)
            frames += b.F
            scenes += 1
            if time.perf_counter() - t0 > budget_s:
                break
        dt = time.perf_counter() - t0
    return dict(value=frames / dt, unit="frames/s", cores=1, kind="port",
                sample=f"{scenes} scenes x {b.F} frames of the same workload "
                       f"(float64 NumPy oracle, 1 thread, {dt:.1f} s)")


def time_train(args, params, t, dev, dist, S, F, world):
    """--mode train: the same step plus loss gradient, ONE
    all-reduce of the flat [P + 2] gradient buffer across ranks (RCCL under
    the nccl backend) and the RMSProp update (multimodaltraj_2_amd/train_step.py).
    Timed like the reference-mode step: barrier + synchronize on both sides,
    max over ranks."""
    from multimodaltraj_2_amd.train_step import TrainStep
    step = TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    for _ in range(args.warmup):
        step.run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        g = step.run()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if dist is not None:
        e = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        el = float(e.item())
    gl = g.double().cpu().numpy()
    return {"metric": "frames/sec (obs=8,pred=12) g2k_lstm_mcr train step + L2 loss gradient + "
                      "gradient all-reduce + RMSProp update",
            "value": S * F * world * args.steps / el, "unit": "frames/s",
            "ms_per_step": el / args.steps * 1e3, "allreduce_bytes": int(g.numel() * 4),
            "loss_per_prediction_last_step": float(gl[-2] / max(gl[-1], 1.0)),
            "optimizer": "RMSProp lr 0.005 decay 0.95, global-norm clip 10 (argParser.py:38-47)"}


def load_pmc(config):
    p = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="eth_hotel_synth", choices=sorted(CONFIGS))
    ap.add_argument("--scenes", type=int, default=0, help="override scenes per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-train", action="store_true", help="skip the --mode train timing")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    cfg = dict(CONFIGS[args.config])
    if args.config in ("eth_ucy_loo_kfold4", "dense_crowd"):
        cfg["S"] = cfg["S"] // 8          # 128 scenes per GPU
    S = args.scenes or cfg["S"]
    Nmax, H, F = cfg["Nmax"], cfg["H"], FRAMES_PER_SCENE
    b = make_batch(S, Nmax, H, F=F, seed=1 + rank)
    params = fs.init_params(Nmax, seed=0, device=dev)
    t = b.to_device(dev)
    out = fs.StepOutputs(pred=torch.empty((S, F, 24, Nmax), device=dev),
                         h=torch.empty((S, 16, H), device=dev),
                         metrics=torch.empty((S, 8), device=dev))

    # one validated launch bound to the resident buffers; each step is one C call
    plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                       t["h0"], out=out)
    step = plan.run

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # reference mode: replicas only; the ADE/FDE numerators are summed across
    # ranks once at the end, outside the timed region
    tot = out.metrics.double().sum(dim=0)
    if dist is not None:
        e = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        dist.all_reduce(tot)

    # dominant-kernel duration: HIP events on the stream the kernel runs on
    stream = torch.cuda.current_stream()
    reps = max(20, min(args.steps, 200))
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(reps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    kern_s = ev0.elapsed_time(ev1) / 1e3 / reps

    frames_total = S * F * world
    value = frames_total * args.steps / elapsed
    pbytes = sum(getattr(params, k).numel() * 4 for k in ("Wi", "Wii", "Wv", "bv", "Wr", "Wc", "Wo"))
    abytes = algorithmic_bytes(b, H, pbytes)
    achieved = abytes / kern_s / 1e9
    pmc = load_pmc(args.config)

    train = None if args.no_train else time_train(args, params, t, dev, dist, S, F, world)

    if rank == 0:
        cpu = None if args.no_cpu_baseline or world > 1 else \
            cpu_baseline(b, params.numpy(), budget_s=args.cpu_budget)
        m = tot.double().cpu().numpy()
        line = {
            "metric": "frames/sec (obs=8,pred=12) g2k_lstm_mcr train step; ADE/FDE vs reference",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded random-walk ETH-shaped scenes; N(0,1) weights)",
            "config": {"workload": args.config, "scenes_per_gpu": S, "global_scenes": S * world,
                       "frames_per_scene": F, "obs_len": 8, "pred_len": 12, "Nmax": Nmax,
                       "hidden": H, "D": 16, "parallelism": f"dp{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": pmc, "kernel": "g2k_step_fused_f32 (g2k_scene_kernel)",
                         "kernel_us": kern_s * 1e6, "algorithmic_bytes": abytes},
            "cpu_baseline": cpu,
            "ade_fde_all_ranks": {"ADE": float(m[0] / max(m[1], 1)),
                                  "FDE_frob_per_frame": float(np.sqrt(m[2]) / max(m[5], 1))},
            "train_mode": train,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
