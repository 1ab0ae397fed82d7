"""Data parallelism over scene batches.

Scenes are independent (no cross-scene term in a1-a9), so every rank owns a
contiguous shard of scenes and runs the HIP step on it with no data-path
collective ("replicas only").  The only exchange is the sum of the ADE/FDE
numerators and counts, once per reporting interval — one tiny all-reduce
(RCCL on ROCm when the backend is "nccl", gloo on CPU).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_scenes(total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous [start, stop) of ``total`` scenes for ``rank`` (sizes differ
    by at most one)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} / world {world}")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def reduce_metrics(metrics: torch.Tensor, group=None) -> torch.Tensor:
    """Per-scene metric rows [S, 8] -> the all-rank sum [8] (float64).
    Field order: see frame_step.METRIC_FIELDS."""
    tot = metrics.to(torch.float64).sum(dim=0)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    return tot


def global_errors(tot: torch.Tensor):
    """(ADE, FDE) over everything summed by reduce_metrics: ADE = mean of the
    per-(frame, pedestrian) spectral ade_i (train.py:648-669); FDE = Frobenius
    norm of the stacked fde vectors over the number of frames (train.py:674)."""
    t = tot.double().cpu()
    cnt = float(t[1])
    if cnt <= 0:
        return float("nan"), float("nan")
    return float(t[0] / cnt), float(torch.sqrt(t[2]) / max(float(t[5]), 1.0))


def allreduce_grad(buf: torch.Tensor, group=None, force: bool = False) -> torch.Tensor:
    """Train mode: sum the flat [P + 2] buffer (gradient
    sums, loss, count) over ranks in place — one collective per step; every
    rank then applies the same update (train_step.TrainStep).  ``force``
    issues the collective on a one-rank group too (the multi-rank structure
    measured and graph-captured on one GPU)."""
    if dist.is_available() and dist.is_initialized() and (force or dist.get_world_size(group) > 1):
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def reap_pending_work(group=None) -> None:
    """Before capturing a collective into a HIP graph: synchronize, then block
    until the process group's watchdog thread holds no eager Work.

    Why (the r7m abort): ProcessGroupNCCL's watchdog polls every
    eager Work it holds with ``hipEventQuery`` on the Work's end event, which
    was recorded on the group's RCCL stream.  A captured collective puts that
    same RCCL stream into capture mode (it waits on the capturing stream), and
    HIP answers a query of an event recorded on a stream that is capturing
    with hipErrorCapturedEvent — the watchdog treats that as fatal (SIGABRT).
    Captured Works are never handed to the watchdog, so the race exists only
    for eager Works still listed when a capture starts (the warm-up step, a
    barrier, a metric all-reduce: reaped ~100 ms after they finish).  This
    torch build's capture_begin no longer waits for them, so we do:
    ``ProcessGroup._wait_for_pending_works`` returns once the watchdog's list
    is empty, and the caller issues no eager collective until the capture
    ends.  A no-op without a process group or on a backend with no watchdog
    (gloo)."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    pg = group if group is not None else dist.group.WORLD
    if dist.get_backend(pg) != "nccl":
        return
    torch.cuda.synchronize()
    pg._wait_for_pending_works()
