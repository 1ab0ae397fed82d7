"""Real ETH/UCY scenes, many distinct ones per launch (BASELINE.json config 3's
workload on the reference's data).

A scene is what sample.py builds for one batch (sample.py:138-164): the
DataLoader's next_step from a frame pointer (load_traj.py:153-224), a FRESH
online graph at framenum 0 (networkx_graph.py:30-73), the time slice of every
node's position list (all P pedestrians of the window, not train.py's node
slice, which is empty after a dataset's first batch) and each node's own 12
targets.  The step runs train.py's frame loop over it (train.py:197): n_frames
= len(batch), the same window every frame (stride 0), the batch's targets every
frame.

Distinct windows: the reference's sample walk visits the pointers seed +
136 j (17 passes of 8 frames per next_step); the same next_step from every
pointer seed + 8 m (m = 0, 1, ...) gives every distinct window of a dataset.
Scenes are taken round-robin over the datasets, m ascending, keeping those
with 2 <= P <= Nmax pedestrians (train.py:86-90 skips fewer than two).

The walk is planned natively (csrc/g2k_walk.cpp, TrajIndex.sample_scenes:
CSV column per window slot and per target step) and expanded on the device by
one g2k_scene_gather_f32 launch from the splits' positions and vislets held in
HBM — no per-scene Python.  Data: the CSVs under a data root
(load_traj.DATA_DIRS) or raw CSV arrays handed in by the caller.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from types import SimpleNamespace

import numpy as np

from .load_traj import DATA_DIRS, DataLoader

DATASETS = {"eth_hotel": 0, "zara01": 2, "zara02": 3, "ucy_univ": 4}   # load_traj.DATA_DIRS index
ARGS = SimpleNamespace(batch_size=16, seq_length=12, pred_len=12, obs_len=8)


def fold_datasets(leave_dataset):
    """train.py:38-39: the training datasets of a leave-one-out fold
    ({2, 3, 4, 5} minus the left-out one; 5, town_center.csv, is absent from the
    reference's data) plus ETH hotel (config 3 is "ETH+UCY")."""
    keep = ({2, 3, 4, 5} - {int(leave_dataset)}) | {0}
    return [n for n, i in DATASETS.items() if i in keep]


def load_raw(names, data_root):
    """Raw CSV arrays (load_traj.py:124) of the named datasets under data_root."""
    out = {}
    for n in names:
        dl = DataLoader(ARGS, datasets=[0, 1, 2, 3, 4, 5], start=DATASETS[n], sel=0,
                        data_root=data_root)
        out[n] = dl.raw_data
    return out


class SceneSource:
    """One dataset as the reference's sample.py walks it: the training split's
    bounds (load_traj.py:133-139, 163) over the frame dict the reference reads
    (the whole CSV for the shipped datasets, load_traj.py:95-112); its native
    walk index and the fp32 position / vislet rows of the dict's columns (the
    vislet slice sample.py:184 reads starts at column 0, shared by both)."""

    def __init__(self, name, raw_data, frame_dict=None):
        self.name = name
        self.loader = DataLoader(ARGS, raw_data=raw_data, frame_dict=frame_dict)
        src = self.loader.dict_data
        self.xy = np.ascontiguousarray(np.stack([src[2], src[3]], axis=1), dtype=np.float32)
        self.vis = (np.ascontiguousarray(src[4:6], dtype=np.float32) if src.shape[0] >= 6 else None)
        self.cols = self.xy.shape[0]
        seed, fmax = float(self.loader.seed), float(self.loader._fmax)
        self.pointers = seed + self.loader.diff * np.arange(int((fmax - seed) // self.loader.diff) + 1)
        # columns holding equal (x, y) values share one id (content keys compare values)
        _, canon = np.unique(self.xy.view(np.int64).reshape(-1), return_inverse=True)
        self.canon = np.append(canon.astype(np.int32), -1)          # canon[-1] = -1
        self._plan = None
        self._cap = None

    def plan(self, count=None, nmax_cap=96):
        """Plans of the first ``count`` pointers (all: None), cached and
        extended on demand: the native sample_scenes output, plus a content key
        per plan (scenes from different pointers can coincide where a pointer
        falls on an empty frame)."""
        count = len(self.pointers) if count is None else min(int(count), len(self.pointers))
        have = 0 if self._plan is None else len(self._plan["n_nodes"])
        if self._cap not in (None, nmax_cap):
            have, self._plan = 0, None
        if count > have:
            new = self.loader.index.sample_scenes(self.pointers[have:count], nmax_cap)
            old = self._plan
            self._plan = new if old is None else {
                k: np.concatenate([old[k], new[k]]) for k in new if k != "content"}
            # content keys over the WHOLE cached plan: the exact fallback of
            # _row_keys numbers rows within one call, so keys of separate
            # extensions must not be mixed
            p = self._plan
            w = max(1, int(p["n_nodes"].max(initial=0)))        # slots >= P are empty (-1)
            p["content"] = _row_keys(self.canon[p["pos_col"][:, :, :w]],
                                     self.canon[p["tgt_col"][:, :w]])
            self._cap = nmax_cap
        return {k: v[:count] for k, v in self._plan.items()}


_HASH = np.random.default_rng(0x9e3779b9).integers(1, 1 << 63, (2, 8 * 256 + 256 * 12),
                                                     dtype=np.uint64) | np.uint64(1)


def _row_keys(pos_col, tgt_col):
    """One 64-bit key per plan row (pos_col [n, 8, w], tgt_col [n, w, 12] of
    canonical column ids, -1 = empty, any w >= the rows' P): equal rows, equal
    keys.  A
    multiply-add hash of (id + 1) per slot with a fixed multiplier per slot
    (t, n) / (n, k), so the empty slots add nothing and the key does not
    depend on how many slots are looked at; rows that share a key and differ
    (never seen) fall back to exact keys by value."""
    n, _, w = pos_col.shape
    pc = (pos_col[:, :, :w].astype(np.int64) + 1).view(np.uint64)
    tc = (tgt_col[:, :w, :].astype(np.int64) + 1).view(np.uint64)
    mp = _HASH[0, :8 * 256].reshape(8, 256)[:, :w]
    mt = _HASH[1, :256 * 12].reshape(256, 12)[:w]
    with np.errstate(over="ignore"):
        key = ((pc * mp).sum(axis=(1, 2), dtype=np.uint64)
               + (tc * mt).sum(axis=(1, 2), dtype=np.uint64))
    u, first, inv = np.unique(key, return_index=True, return_inverse=True)
    if len(u) < len(key):                      # equal keys: equal rows?
        f = first[inv.reshape(-1)]
        if not (np.all(pc == pc[f], axis=(1, 2)) & np.all(tc == tc[f], axis=(1, 2))).all():
            rows = np.concatenate([pc.reshape(n, -1), tc.reshape(n, -1)], axis=1)
            _, key = np.unique(rows, axis=0, return_inverse=True)
            key = key.reshape(-1).astype(np.uint64) | np.uint64(1 << 63)
    return key


@dataclass
class RealPlan:
    """S scenes' index plans over the concatenated splits of their datasets."""
    names: list            # dataset of each scene
    pointers: np.ndarray   # [S] frame pointer of each scene
    pos_col: np.ndarray    # [S, 8, Nmax] int32 (global column, -1 = zero slot)
    tgt_col: np.ndarray    # [S, Nmax, 12] int32
    n_active: np.ndarray   # [S] int32 = P
    n_frames: np.ndarray   # [S] int32 = len(batch)
    xy: np.ndarray         # [C, 2] f32, all datasets' columns
    vis: np.ndarray        # [2, C] f32 (zeros for ETH, Q14)
    vis_off: np.ndarray    # [S] int32: the dataset's first column (slice vislet[:, 0:P])

    @property
    def S(self):
        return int(self.n_active.shape[0])

    @property
    def Nmax(self):
        return int(self.pos_col.shape[2])

    def to_device(self, device, F=None, stream=None):
        """The step's inputs in HBM by one g2k_scene_gather_f32 launch:
        dict(pos [S, 8, Nmax, 2], vislet, targets [S, F, Nmax, 12, 2],
        n_active, n_frames, ped_mask)."""
        import torch
        from . import _lib
        lib = _lib.load()
        F = int(F or self.n_frames.max())
        S, N = self.S, self.Nmax
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        xy, vis, pc, tc = t(self.xy), t(self.vis), t(self.pos_col), t(self.tgt_col)
        voff, nact, nfr = t(self.vis_off), t(self.n_active), t(self.n_frames)
        out = dict(pos=torch.empty((S, 8, N, 2), device=device),
                   vislet=torch.empty((S, 2, N), device=device),
                   targets=torch.empty((S, F, N, 12, 2), device=device),
                   ped_mask=torch.empty((S, N), dtype=torch.uint8, device=device),
                   n_active=nact, n_frames=nfr)
        s = stream if stream is not None else torch.cuda.current_stream(device)
        rc = lib.g2k_scene_gather_f32(xy.data_ptr(), vis.data_ptr(), int(self.xy.shape[0]),
                                      pc.data_ptr(), tc.data_ptr(), voff.data_ptr(),
                                      nact.data_ptr(), S, F, N, out["pos"].data_ptr(),
                                      out["vislet"].data_ptr(), out["targets"].data_ptr(),
                                      out["ped_mask"].data_ptr(), ctypes.c_void_p(s.cuda_stream))
        _lib.check("g2k_scene_gather_f32", rc)
        out["_keep"] = (xy, vis, pc, tc, voff)
        return out

    def host(self, F=None):
        """The same tensors on the host (numpy), for the oracle and the CPU
        baseline: pos, vislet, targets, ped_mask."""
        F = int(F or self.n_frames.max())
        S, N = self.S, self.Nmax
        lane = np.arange(N)[None, :]
        act = lane < self.n_active[:, None]                                 # [S, N]
        pc = np.where(act[:, None, :], self.pos_col, -1)
        pos = np.where(pc[..., None] >= 0, self.xy[np.maximum(pc, 0)], 0).astype(np.float32)
        c = self.vis_off[:, None] + lane
        vislet = np.where(act[:, None, :], self.vis[:, np.minimum(c, self.vis.shape[1] - 1)]
                          .transpose(1, 0, 2), 0).astype(np.float32)
        tc = np.where(act[:, :, None], self.tgt_col, -1)
        tg = np.where(tc[..., None] >= 0, self.xy[np.maximum(tc, 0)], 0).astype(np.float32)
        mask = (act & (tc >= 0).all(axis=2)).astype(np.uint8)
        targets = np.ascontiguousarray(np.broadcast_to(tg[:, None], (S, F, N, 12, 2)))
        return dict(pos=pos, vislet=vislet, targets=targets, ped_mask=mask,
                    n_active=self.n_active.copy(), n_frames=self.n_frames.copy())


def plan_scenes(S, raw_by_name, nmax=None, min_peds=2, sources=None):
    """S distinct scenes round-robin over the datasets of ``raw_by_name``
    ({name: raw CSV array}); Nmax = ``nmax`` or the largest P rounded up to 16
    (scenes with P > nmax are left out)."""
    sources = sources or [SceneSource(n, raw_by_name[n]) for n in raw_by_name]
    cap = max(96, nmax or 0)
    want = -(-S // len(sources)) + 8
    while True:
        plans = [src.plan(want, cap) for src in sources]
        pools = []
        for src, p in zip(sources, plans):
            P = p["n_nodes"]
            ok = (P >= min_peds) & (P <= (nmax or cap))
            _, first = np.unique(p["content"], return_index=True)   # distinct contents only
            keep = np.zeros(len(P), bool)
            keep[first] = True
            pools.append(np.flatnonzero(ok & keep))
        if sum(len(x) for x in pools) >= S or all(len(p["n_nodes"]) == len(src.pointers)
                                                  for src, p in zip(sources, plans)):
            break
        want *= 2
    avail = sum(len(x) for x in pools)
    if avail < S:
        raise ValueError(f"only {avail} distinct scenes with {min_peds} <= P <= {nmax or cap} "
                         f"in {[s.name for s in sources]}, {S} requested")
    # round-robin over the datasets: the r-th scene of every dataset, then the (r+1)-th
    rank = np.concatenate([np.arange(len(p)) for p in pools])
    dset = np.concatenate([np.full(len(p), d) for d, p in enumerate(pools)])
    idx = np.concatenate(pools)
    order = np.lexsort((dset, rank))[:S]
    dsel, jsel = dset[order], idx[order]
    P = np.empty(S, np.int32)
    nfr = np.empty(S, np.int32)
    for d in range(len(sources)):
        m = dsel == d
        P[m] = plans[d]["n_nodes"][jsel[m]]
        nfr[m] = plans[d]["n_keys"][jsel[m]]
    N = int(nmax or max(16, -(-int(P.max()) // 16) * 16))
    base = np.cumsum([0] + [s.cols for s in sources]).astype(np.int32)
    pos_col = np.full((S, 8, N), -1, np.int32)
    tgt_col = np.full((S, N, 12), -1, np.int32)
    w = min(N, cap)
    for d in range(len(sources)):
        m = np.flatnonzero(dsel == d)
        pc = plans[d]["pos_col"][jsel[m]][:, :, :w]
        tc = plans[d]["tgt_col"][jsel[m]][:, :w]
        pos_col[m, :, :w] = np.where(pc >= 0, pc + base[d], -1)
        tgt_col[m, :w] = np.where(tc >= 0, tc + base[d], -1)
    xy = np.concatenate([s.xy for s in sources], axis=0)
    vis = np.concatenate([s.vis if s.vis is not None else np.zeros((2, s.cols), np.float32)
                          for s in sources], axis=1)
    return RealPlan(names=[sources[d].name for d in dsel],
                    pointers=np.array([sources[d].pointers[j] for d, j in zip(dsel, jsel)]),
                    pos_col=pos_col, tgt_col=tgt_col, n_active=P, n_frames=nfr,
                    xy=xy, vis=vis, vis_off=base[dsel].astype(np.int32))


def count_scenes(raw_by_name, nmax=None, min_peds=2):
    """How many distinct scenes plan_scenes can take from these datasets."""
    n = 0
    cap = max(96, nmax or 0)
    for name, raw in raw_by_name.items():
        p = SceneSource(name, raw).plan(None, cap)
        P = p["n_nodes"]
        ok = (P >= min_peds) & (P <= (nmax or cap))
        _, first = np.unique(p["content"], return_index=True)
        keep = np.zeros(len(P), bool)
        keep[first] = True
        n += int((ok & keep).sum())
    return n


def data_root_raw(data_root, names):
    """{name: raw CSV array} from a data root laid out as the reference's
    data/ directory (load_traj.py:25-33)."""
    missing = [n for n in names if not os.path.isdir(os.path.join(data_root, DATA_DIRS[DATASETS[n]]))]
    if missing:
        raise FileNotFoundError(f"{missing} not under {data_root}")
    return load_raw(names, data_root)
