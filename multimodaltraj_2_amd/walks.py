"""The reference's batch walks over one dataset, as plans for the HIP step.

The reference's entry points interleave their data walk with the per-frame
TF body; here the data side runs first and yields one record per iteration of
the reference's batch loop, with everything the fused step and the logs need
(the window of the batch's node slice, the vislet offset, the frame count, the
targets).  The control flow is the reference's, line by line:

* ``train_walk`` — train.py:53-90 (graph per dataset, batch setup and its
  batch_v checks: no nodes or one node -> ``reset_data_pointer(); break``,
  zero nodes proceed), :197 (the frame loop leaves ``frame`` at the batch's
  last key), :278-299 (the next batch's ConstructGraph and checks; the top of
  the loop then builds the graph a second time, :74), :59-67 and :353 (epochs;
  an empty first batch resets the pointer without ending the epoch).
* ``valid_walk`` — train.py:371-445, 556, 681 (fresh graph, frame = 1,
  framenum = the returned frame pointer, the pointer set to the batch's last
  key after each batch).
* ``sample_walk`` — sample.py:125-164 (fresh graph per batch, framenum 0, time
  slice).

Frame keys are cast to int where the reference uses them as indices (quirk
Q9).  Pinned against replays of the reference's own load_traj/networkx_graph
over every batch (tests/golden/walk_*.npz, tools/ref_walks.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import networkx_graph as nxg


@dataclass
class WalkBatch:
    """One iteration of a reference batch loop."""
    index: tuple                 # (epoch, b) / (vb,) / (b,)
    frame: float                 # the `frame` value at the loop's top (slice start)
    batch: dict                  # x_batch of next_step
    target_traj: dict            # targets of next_step
    node_ids: np.ndarray         # graph node ids after the loop's ConstructGraph
    npl: np.ndarray              # their node_pos_list [P, 8, 2]
    n: int                       # num_nodes (-1: the reference breaks here)
    window: np.ndarray | None    # [8, n, 2]: window[t, i] = the slice's node i, row t
    vis_off: int = 0             # vislet column offset of the slice
    frame_after: float = 0.0     # `frame` after the batch's frame loop
    outcome: str = "next"        # what ended the iteration
    fp: float = 0.0              # frame pointer returned by next_step (validation)
    extra: dict = field(default_factory=dict)

    @property
    def n_frames(self) -> int:
        return len(self.batch)


def _snapshot(graph_t):
    npl_d = graph_t.get_node_attr("node_pos_list")
    ids = np.array(list(npl_d.keys()), dtype=np.int64)
    npl = np.array(list(npl_d.values()), dtype=np.float64).reshape(-1, 8, 2)
    return ids, npl


def _node_slice(npl, frame, obs_len):
    """train.py:77-90: (n, window) of the node slice [frame:frame+obs_len];
    n = -1 where the reference breaks (no nodes, or one node: squeeze leaves
    a 1-d batch_v and .shape[1] raises IndexError)."""
    if npl.shape[0] == 0:
        return -1, None
    sl = npl[frame:frame + obs_len]
    if sl.shape[0] == 1:
        return -1, None
    return sl.shape[0], np.ascontiguousarray(np.transpose(sl, (1, 0, 2)))


def train_walk(loader, args, epochs, frame=1, graph=None, counters=None, epoch0=0):
    """train.py:53-353 for one dataset.  Yields WalkBatch records (n >= 0: the
    frame loop runs over the batch; n = -1: the loop broke there) and, at each
    epoch end, the string "epoch_end".  ``counters`` (dict with num_targets,
    num_end_targets) is updated as train.py:255-259 does; ``frame`` carries
    in and its final value is in ``counters['frame']``; the epoch counter runs
    from ``epoch0`` to ``epochs`` (train.py sets e = 0 once per left-out
    dataset, :29, so a later dataset of the fold starts where the first ended)."""
    graph = graph or nxg.online_graph(args)
    counters = counters if counters is not None else {}
    counters.setdefault("num_targets", 0)
    counters.setdefault("num_end_targets", 0)
    loader.reset_data_pointer()                                   # :56
    counters["frame"] = float(frame)
    e, guard = epoch0, 0
    while e < epochs:                                             # :59
        guard += 1
        if guard > 10 * (epochs - epoch0) + 100:
            raise RuntimeError("train walk does not advance (no non-empty batch)")
        batch, target_traj, _ = loader.next_step()                # :61
        if len(batch) == 0:                                       # :63-67
            loader.reset_data_pointer()
            continue
        for b in range(loader.num_batches):                       # :71
            fi = int(frame)
            g = graph.ConstructGraph(current_batch=batch, framenum=fi, future_traj=target_traj)
            ids, npl = _snapshot(g)                               # :74-76
            n, window = _node_slice(npl, fi, args.obs_len)
            rec = WalkBatch((e, b), float(frame), batch, target_traj, ids, npl, n, window,
                            vis_off=fi)
            if n < 0:                                             # :80-83, 86-90
                rec.outcome = "reset_break"
                yield rec
                loader.reset_data_pointer()
                break
            for frame in batch:                                   # :197
                counters["num_targets"] += n                      # :255
                counters["num_end_targets"] += min(max(n - 1, 0), len(target_traj))   # :257-259
            rec.frame_after = float(frame)
            batch, target_traj, _ = loader.next_step()            # :278
            fi = int(frame)
            g = graph.ConstructGraph(current_batch=batch, framenum=fi, future_traj=target_traj)
            nxt_ids, nxt_npl = _snapshot(g)                       # :280-282
            if nxt_npl.shape[0] == 0:                             # :284-285
                rec.outcome = "break"
            elif _node_slice(nxt_npl, fi, args.obs_len)[0] < 0:   # :286-299
                rec.outcome = "reset_break"
            counters["frame"] = float(frame)
            yield rec
            if rec.outcome == "reset_break":
                loader.reset_data_pointer()
            if rec.outcome != "next":
                break
        counters["frame"] = float(frame)
        yield "epoch_end"                                         # :348-353
        e += 1


def valid_walk(loader, args, start_pointer=0):
    """train.py:371-445, 556, 681: yields WalkBatch records; the reason the
    walk ended is in the last record's ``extra['end']`` or, when no batch was
    seen, raised as StopIteration's value."""
    graph = nxg.online_graph(args)                                # :374
    loader.reset_data_pointer(valid=True, frame_pointer=start_pointer)   # :377
    vfp = int((loader.len - int(loader.max * .7)) / loader.val_max)      # :408-409
    vnb = int(loader.val_max / loader.batch_size)                        # :411
    loader.valid_frame_pointer, loader.valid_num_batches = vfp, vnb
    frame = 1                                                     # :392
    for vb in range(vnb):                                         # :423
        batch, target_traj, fp = loader.next_step()               # :426
        if len(batch) == 0:                                       # :428-429
            return "empty"
        g = graph.ConstructGraph(current_batch=batch, framenum=int(fp), future_traj=target_traj)
        ids, npl = _snapshot(g)                                   # :431-432
        if npl.shape[0] == 0:                                     # :434-435
            return "no_nodes"
        n, window = _node_slice(npl, int(frame), args.obs_len)    # :437-445
        rec = WalkBatch((vb,), float(frame), batch, target_traj, ids, npl, n, window,
                        vis_off=vfp, fp=float(fp))
        if n < 0:                                                 # :445 (uncaught IndexError)
            rec.outcome = "crash_n1"
            yield rec
            return "crash_n1"
        for frame in batch:                                       # :556
            pass
        loader.frame_pointer = frame                              # :681
        rec.frame_after = float(frame)
        yield rec
    return "exhausted"


def sample_walk(loader, args, offset=0, max_batches=None):
    """sample.py:125-164 from frame pointer seed + obs_len*offset: one fresh
    graph per batch, ConstructGraph(framenum=0), the time slice (all P nodes)."""
    loader.reset_data_pointer()                                   # :125
    loader.frame_pointer += loader.diff * offset
    b = 0
    while max_batches is None or b < max_batches:
        fp0 = float(loader.frame_pointer)
        x_batch, y_batch, _ = loader.next_step()                  # :140
        if len(x_batch) == 0:                                     # :146-147
            return
        g = nxg.online_graph(args).ConstructGraph(current_batch=x_batch, framenum=0,
                                                  future_traj=y_batch)   # :150-151
        ids, npl = _snapshot(g)
        window = np.ascontiguousarray(np.transpose(npl, (1, 0, 2)))     # :154 time slice
        tg = g.get_node_attr("targets")
        rec = WalkBatch((b,), 0.0, x_batch, y_batch, ids, npl, len(ids), window, vis_off=0,
                        fp=fp0)
        rec.extra["node_targets"] = [v[0] for v in tg.values()]         # :329
        yield rec
        b += 1
