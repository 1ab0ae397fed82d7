"""Real-data batches -> HIP step inputs (the caller side of the hot path,
train.py:71-196 / sample.py:138-211).

One reference batch (16 frame keys of ``DataLoader.next_step``) becomes one
scene: the position window [8, N, 2] of the batch's online graph (node slice
of train.py:78 or time slice of sample.py:154), the frame loop of
train.py:197 as ``n_frames = len(batch)`` frames over that same window
(stride 0: the reference feeds identical inputs to every frame of a batch),
the vislet slice of train.py:182, and per prediction row the target of the
row's pedestrian key in ``target_traj`` insertion order (validation pairing,
train.py:640), truncated to pred_len (targets are 12k long, quirk Q11).
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
                pred_len=12):
    npl = np.array(list(graph_t.get_node_attr("node_pos_list").values()), dtype=np.float64)
    npl = npl.reshape(-1, 8, 2)
    fr = int(frame)
    window = nxg.scene_tensors(npl, obs_len=obs_len, frame=fr if mode == "train" else 0, mode=mode)
    n = window.shape[1]
    off = fr if mode == "train" else 0
    vis = np.zeros((2, n))
    src = loader.vislet[:, off:off + n]
    vis[:, :src.shape[1]] = src
    keys = list(target_traj.keys())
    targets = np.zeros((n, pred_len, 2))
    mask = np.zeros(n, bool)
    for i in range(min(n, len(keys))):
        t = np.asarray(target_traj[keys[i]], dtype=np.float64).reshape(-1, 2)
        if len(t) >= pred_len:
            targets[i] = t[:pred_len]
            mask[i] = True
    return RealScene(window, vis, targets, mask, len(batch), keys)


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
