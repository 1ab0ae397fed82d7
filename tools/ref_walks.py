"""Replays of the reference's batch walks, for fixture generation only.

Runs in the build container, where /root/reference exists: it drives the
reference's OWN data modules (load_traj.DataLoader.next_step,
networkx_graph.online_graph.ConstructGraph / get_node_attr) through the
control flow of the reference's entry points, which cannot be imported (they
need TensorFlow 1.x), restated here line by line:

  train_walk  train.py:56-90 (epoch start, batch setup), :197 (the frame loop
              leaves `frame` at the batch's last key), :257-276 (counters),
              :278-299 (next batch: the second ConstructGraph of every batch)
              and :353 (epoch end), for ONE dataset of the fold;
  valid_walk  train.py:371-445 + :556 + :681 (fresh graph, frame = 1,
              framenum = the returned frame pointer, pointer := last key);
  sample_walk sample.py:138-164 (fresh graph per batch, framenum 0, time
              slice), from the data seed or from seed + 8k (the build's
              distinct-window supply: the same next_step from a shifted
              pointer).

Every walk returns a list of per-batch records (plain dicts of numpy arrays
and ints).  The TF arithmetic of the loop bodies is not replayed: only what
the data side hands to it.  Nothing here is imported by the product.
"""
from __future__ import annotations

import hashlib

import numpy as np


def digest(*arrays) -> str:
    h = hashlib.sha1()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def _targets_record(target_traj, first=12, max_keys=None):
    """The target dict of one batch: keys (insertion order), list lengths,
    the first 12 points of the first ``max_keys`` keys (all a pairing can
    read: the lists are 12 copies per draw, quirk Q11) and a digest of all
    lists."""
    keys = list(target_traj.keys())
    lens = np.array([len(target_traj[k]) for k in keys], dtype=np.int64)
    hk = keys if max_keys is None else keys[:max_keys]
    head = np.zeros((len(hk), first, 2))
    for j, k in enumerate(hk):
        t = np.asarray(target_traj[k], dtype=np.float64).reshape(-1, 2)[:first]
        head[j, :len(t)] = t
    full = (np.concatenate([np.asarray(target_traj[k], np.float64).reshape(-1, 2) for k in keys])
            if keys else np.zeros((0, 2)))
    return dict(tkeys=np.array(keys, dtype=np.int64), tlens=lens, thead=head,
                tdigest=digest(full))


def _graph_record(graph_t):
    npl_d = graph_t.get_node_attr(param="node_pos_list")
    ids = np.array(list(npl_d.keys()), dtype=np.int64)
    npl = np.array(list(npl_d.values()), dtype=np.float64).reshape(-1, 8, 2)
    return ids, npl


def train_walk(dl, graph_mod, args, epochs):
    """train.py:56-353 for the first dataset of a fold (``e``, ``frame`` and the
    counters start at 0 / 1 / 0, train.py:29-36).  Records one entry per
    batch-loop iteration (the ConstructGraph of train.py:74), with the outcome
    of its batch_v checks, and the epoch-level events."""
    graph = graph_mod.online_graph(args)                      # :53
    dl.reset_data_pointer()                                   # :56
    frame = 1                                                 # :34
    num_targets = num_end_targets = 0                         # :35-36
    n_fde = 0
    e = 0
    recs, events = [], []
    guard = 0
    while e < epochs:                                         # :59
        guard += 1
        if guard > 10 * epochs + 100:
            raise RuntimeError("train walk does not advance")
        batch, target_traj, _ = dl.next_step()                # :61
        if len(batch) == 0:                                   # :63-67
            events.append(("empty_reset", e))
            dl.reset_data_pointer()
            continue
        for b in range(dl.num_batches):                       # :71
            fi = int(frame)                                   # float key as index: Q9
            graph_t = graph.ConstructGraph(current_batch=batch, framenum=fi,
                                           future_traj=target_traj)   # :74
            ids, npl = _graph_record(graph_t)
            rec = dict(e=e, b=b, frame=float(frame), keys=np.array(list(batch.keys()), np.float64),
                       node_ids=ids, npl_digest=digest(ids, npl), P=len(ids))
            rec.update(_targets_record(target_traj, max_keys=8))
            bv = list(graph_t.get_node_attr(param="node_pos_list").values())
            outcome = None
            if len(np.array(bv).shape) > 1:                   # :77-79
                sl = np.array(bv)[fi:fi + args.obs_len]
                rec["window"] = np.ascontiguousarray(np.transpose(sl, (1, 0, 2))) \
                    if sl.ndim == 3 else np.zeros((8, 0, 2))
                bv = np.linalg.norm(sl, axis=2).squeeze()
            else:
                outcome = "reset_break"                       # :80-83
            if outcome is None:
                bv = np.transpose(bv)                         # :85
                try:
                    num_nodes = bv.shape[1]                   # :86-90
                except IndexError:
                    outcome = "reset_break"
            if outcome is not None:
                rec["outcome"] = outcome
                rec["n"] = -1
                recs.append(rec)
                dl.reset_data_pointer()
                break
            rec["n"] = int(num_nodes)
            rec["batch_v"] = np.asarray(bv, np.float64)
            rec["vis_off"] = float(frame)                     # :182 vislet[:, frame:frame+N]
            for frame in batch:                               # :197
                num_targets += num_nodes                      # :255
                for i, itr in zip(range(1, num_nodes), iter(target_traj)):   # :257
                    num_end_targets += 1
                    if i in target_traj:
                        n_fde += 1
            rec["frame_after"] = float(frame)
            rec["num_targets"], rec["num_end_targets"], rec["n_fde"] = (
                num_targets, num_end_targets, n_fde)
            batch, target_traj, _ = dl.next_step()            # :278
            fi = int(frame)
            graph_t = graph.ConstructGraph(current_batch=batch, framenum=fi,
                                           future_traj=target_traj)   # :280
            bv = list(graph_t.get_node_attr(param="node_pos_list").values())
            tail = "next"
            if len(bv) == 0:                                  # :284-285
                tail = "break"
            elif len(np.array(bv).shape) > 1:                 # :286-288
                bv = np.linalg.norm(np.array(bv)[fi:fi + args.obs_len], axis=2).squeeze()
                bv = np.transpose(bv)
                try:
                    bv.shape[1]                               # :295-299
                except IndexError:
                    tail = "reset_break"
            else:
                tail = "reset_break"                          # :289-292
            rec["outcome"] = tail
            recs.append(rec)
            if tail == "reset_break":
                dl.reset_data_pointer()
            if tail != "next":
                break
        events.append(("epoch_end", e, n_fde))                # :348-353 (np.stack(fde) needs n_fde > 0)
        e += 1
    return recs, events


def valid_walk(dl, graph_mod, args, start_pointer, keep_targets=False):
    """train.py:371-445, 556, 681: the validation leg's data side from
    ``start_pointer`` (the reference: 0, reset_data_pointer(valid=True)).
    ``keep_targets``: each record also holds a copy of the batch's target dict
    as next_step returned it (``target_traj``: a fresh dict per call —
    next_step rebinds its empty default argument at the first insertion,
    load_traj.py:208-209 — so a record's copy is that batch's dict only)."""
    graph = graph_mod.online_graph(args)                      # :374
    dl.reset_data_pointer(valid=True, frame_pointer=start_pointer)   # :377
    valid_frame_pointer = int((dl.len - int(dl.max * .7)) / dl.val_max)   # :408-409
    valid_num_batches = int(dl.val_max / dl.batch_size)       # :411
    frame = 1                                                 # :392
    recs = []
    end = "exhausted"
    for vb in range(valid_num_batches):                       # :423
        batch, target_traj, fp = dl.next_step()               # :426
        if len(batch) == 0:                                   # :428-429
            end = "empty"
            break
        graph_t = graph.ConstructGraph(current_batch=batch, framenum=int(fp),
                                       future_traj=target_traj)   # :431 (Q9)
        ids, npl = _graph_record(graph_t)
        rec = dict(vb=vb, frame=float(frame), fp=float(fp),
                   keys=np.array(list(batch.keys()), np.float64), node_ids=ids,
                   npl_digest=digest(ids, npl), P=len(ids), vis_off=float(valid_frame_pointer))
        rec.update(_targets_record(target_traj, max_keys=8))
        if keep_targets:
            rec["target_traj"] = {k: [list(p) for p in v] for k, v in target_traj.items()}
        bv = list(graph_t.get_node_attr(param="node_pos_list").values())
        if len(bv) == 0:                                      # :434-435
            end = "no_nodes"
            break
        if len(np.array(bv).shape) <= 1:                      # :437-442
            end = "flat"
            break
        sl = np.array(bv)[int(frame):int(frame) + args.obs_len]
        rec["window"] = (np.ascontiguousarray(np.transpose(sl, (1, 0, 2))) if len(sl)
                         else np.zeros((8, 0, 2)))
        bv = np.transpose(np.linalg.norm(sl, axis=2).squeeze())
        if bv.ndim < 2:                                       # :445 IndexError (uncaught)
            rec["n"] = -1
            recs.append(rec)
            end = "crash_n1"
            break
        rec["n"] = int(bv.shape[1])
        rec["batch_v"] = np.asarray(bv, np.float64)
        for frame in batch:                                   # :556
            pass
        dl.frame_pointer = frame                              # :681
        rec["frame_after"] = float(frame)
        recs.append(rec)
    return recs, dict(end=end, valid_num_batches=valid_num_batches,
                      valid_frame_pointer=valid_frame_pointer)


def sample_walk(dl, graph_mod, args, offset=0, max_batches=None, keep_targets=False):
    """sample.py:125-164 from frame pointer seed + 8*offset: a fresh graph per
    batch, ConstructGraph(framenum=0), time slice.  Stops at the first empty
    batch (sample.py:146-147) or after ``max_batches`` (sample.py runs
    num_batches).  ``keep_targets``: each record also holds a copy of the
    target dict next_step returned (``target_traj``, see valid_walk)."""
    dl.reset_data_pointer()                                   # :125
    dl.frame_pointer += dl.diff * offset
    frame = 0                                                 # :128
    recs = []
    b = 0
    while max_batches is None or b < max_batches:
        fp0 = float(dl.frame_pointer)
        x_batch, y_batch, _ = dl.next_step()                  # :140
        if len(x_batch) == 0:                                 # :146-147
            break
        graph_t = graph_mod.online_graph(args).ConstructGraph(
            current_batch=x_batch, framenum=frame, future_traj=y_batch)   # :150-151
        ids, npl = _graph_record(graph_t)
        tg = graph_t.get_node_attr(param="targets")           # :329
        tl = np.array([len(v[0]) for v in tg.values()], dtype=np.int64)
        th = np.zeros((len(ids), 12, 2))
        for j, v in enumerate(tg.values()):
            t = np.asarray(v[0], np.float64).reshape(-1, 2)[:12]
            th[j, :len(t)] = t
        recs.append(dict(b=b, fp=fp0, keys=np.array(list(x_batch.keys()), np.float64),
                         node_ids=ids, npl=npl, node_tlens=tl, node_targets=th,
                         P=len(ids)))
        if keep_targets:
            recs[-1]["target_traj"] = {k: [list(p) for p in v] for k, v in y_batch.items()}
        b += 1
    return recs
