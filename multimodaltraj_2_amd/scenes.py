"""Real-data batches -> HIP step inputs (the caller side of the hot path,
train.py:71-196 / sample.py:138-211).

One reference batch (16 frame keys of ``DataLoader.next_step``) becomes one
scene: the position window [8, N, 2] of the batch's online graph (node slice
of train.py:78 or time slice of sample.py:154), the frame loop of
train.py:197 as ``n_frames = len(batch)`` frames over that same window
(stride 0: the reference feeds identical inputs to every frame of a batch),
the vislet slice of train.py:182, and per prediction row the target of the
row's pedestrian key in ``target_traj`` insertion order (validation pairing,
train.py:640) or of the key before it (the training log's pairing,
train.py:257), truncated to pred_len (targets are 12k long, quirk Q11).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import networkx_graph as nxg


@dataclass
class RealScene:
    window: np.ndarray      # [8, N, 2]
    vislet: np.ndarray      # [2, N]
    targets: np.ndarray     # [N, 12, 2]
    mask: np.ndarray        # [N] bool: row has a target
    n_frames: int
    keys: list


def build_scene(batch, target_traj, graph_t, loader, frame, *, mode="train", obs_len=8,
                pred_len=12, pairing="row", vislet_offset=None):
    """One batch -> RealScene.  ``pairing``: "row" — prediction row i takes
    the target of key i (the validation pairing, train.py:640-651); or
    "train_log" — row i >= 1 takes key i - 1 and row 0 none (train.py:257-276
    ``zip(range(1, num_nodes), iter(target_traj))``), a row kept only where
    the reference's ``target_traj[i]`` lookup (pedestrian id i) succeeds.  Rows
    are masked in unless their target is shorter than pred_len (the
    reference's short-target branch, handled on the host by
    train_log_vectors).  ``vislet_offset``: the vislet column slice start
    (train.py:182 frame, :474-475 valid_frame_pointer)."""
    npl = np.array(list(graph_t.get_node_attr("node_pos_list").values()), dtype=np.float64)
    npl = npl.reshape(-1, 8, 2)
    fr = int(frame)
    window = nxg.scene_tensors(npl, obs_len=obs_len, frame=fr if mode == "train" else 0, mode=mode)
    n = window.shape[1]
    off = (fr if mode == "train" else 0) if vislet_offset is None else int(vislet_offset)
    vis = np.zeros((2, n))
    src = loader.vislet[:, off:off + n]
    vis[:, :src.shape[1]] = src
    keys = list(target_traj.keys())
    targets = np.zeros((n, pred_len, 2))
    mask = np.zeros(n, bool)
    if pairing == "row":
        rows = [(i, keys[i]) for i in range(min(n, len(keys)))]
    elif pairing == "train_log":
        rows = [(i, itr) for i, itr in zip(range(1, n), keys) if i in target_traj]
    else:
        raise ValueError(f"pairing {pairing!r}")
    for i, k in rows:
        t = np.asarray(target_traj[k], dtype=np.float64).reshape(-1, 2)
        if len(t) >= pred_len and (pairing == "row" or len(target_traj[i]) >= pred_len):
            targets[i] = t[:pred_len]
            mask[i] = True
    return RealScene(window, vis, targets, mask, len(batch), keys)


def scene_from_record(rec, loader, *, pairing="row", pred_len=12):
    """A walks.WalkBatch (n >= 0) -> RealScene: its window (the node slice of
    train.py:78 / the time slice of sample.py:154), the vislet columns
    [vis_off, vis_off + n) of the split (train.py:182, 527; zero past the
    split's end, where the reference's matmul would fail), and the targets of
    ``pairing`` (see build_scene); n_frames = len(batch)."""
    n = max(int(rec.n), 0)
    window = rec.window if rec.window is not None else np.zeros((8, 0, 2))
    vis = np.zeros((2, n))
    src = loader.vislet[:, rec.vis_off:rec.vis_off + n]
    vis[:, :src.shape[1]] = src
    tt = rec.target_traj
    keys = list(tt.keys())
    targets = np.zeros((n, pred_len, 2))
    mask = np.zeros(n, bool)
    if pairing == "row":
        rows = [(i, keys[i]) for i in range(min(n, len(keys)))]
    elif pairing == "train_log":
        rows = [(i, itr) for i, itr in zip(range(1, n), keys) if i in tt]
    elif pairing == "node":                       # sample.py: each node's own targets
        rows = [(i, None) for i in range(n)]
    else:
        raise ValueError(f"pairing {pairing!r}")
    for i, k in rows:
        seq = rec.extra["node_targets"][i] if k is None else tt[k]
        t = np.asarray(seq, dtype=np.float64).reshape(-1, 2)
        if len(t) >= pred_len and (pairing != "train_log" or len(tt[i]) >= pred_len):
            targets[i] = t[:pred_len]
            mask[i] = True
    return RealScene(np.asarray(window, np.float64).reshape(8, n, 2), vis, targets, mask,
                     rec.n_frames, keys)


def train_log_vectors(pred_path_band, target_traj, pred_len=12):
    """train.py:254-276 for one frame's pred_path_band [2, L, N]: the raw
    difference vectors the training leg logs (train.py:348-351), row i >= 1
    against key i - 1: (euc rows [k, 2] per pair, fde [2] per pair).  Host
    formatting of the kernel's predictions, in the reference's order and with
    its index quirks (the short-target branch reads target_traj[i], the
    pedestrian with id i; a missing id skips the row)."""
    P = np.transpose(np.asarray(pred_path_band, dtype=np.float64), (2, 1, 0))
    euc, fde = [], []
    for i, itr in zip(range(1, P.shape[0]), iter(target_traj)):
        if i not in target_traj:
            continue                                     # KeyError, train.py:274-276
        t = np.asarray(target_traj[itr], dtype=np.float64).reshape(-1, 2)
        if len(target_traj[i]) < pred_len:
            euc.append(P[i][0:len(t)] - t)
            fde.append(P[i][len(t) - 1] - t[len(target_traj[i]) - 1])
        else:
            euc.append(P[i][0:pred_len] - t[0:pred_len])
            fde.append(P[i][pred_len - 1] - t[pred_len - 1])
    return euc, fde


def pack(scenes, H, nmax=None, F=None):
    """Stack RealScenes into padded step tensors (numpy, float32)."""
    S = len(scenes)
    n_need = max([sc.window.shape[1] for sc in scenes] + [1])
    Nmax = nmax or max(4, (n_need + 3) // 4 * 4)
    F = F or max([sc.n_frames for sc in scenes] + [1])
    pos = np.zeros((S, 8, Nmax, 2), np.float32)
    vis = np.zeros((S, 2, Nmax), np.float32)
    tgt = np.zeros((S, F, Nmax, 12, 2), np.float32)
    nact = np.zeros(S, np.int32)
    nfr = np.zeros(S, np.int32)
    pm = np.zeros((S, Nmax), np.uint8)
    for s, sc in enumerate(scenes):
        n = sc.window.shape[1]
        pos[s, :, :n] = sc.window
        vis[s, :, :n] = sc.vislet
        tgt[s, :, :n] = sc.targets[None]
        nact[s] = n
        nfr[s] = sc.n_frames
        pm[s, :n] = sc.mask
    return dict(pos=pos, vislet=vis, targets=tgt, n_active=nact, n_frames=nfr, ped_mask=pm,
                Nmax=Nmax, F=F)
