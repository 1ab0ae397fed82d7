"""Real ETH/UCY scenes packed many to a launch (BASELINE.json config 3, the
leave-one-out k-fold workload, on real data).

train.py walks one dataset's batches in order and carries the hidden state
from batch to batch, so only batches of the SAME dataset are ordered; with
the chain cut (h0 = 0 per batch, --chain_hidden 0) every batch is an
independent scene and any number of them, from any datasets, share one
[S, ...] launch.  Scenes are drawn round-robin over the datasets from each
dataset's own batch walk (load_traj.DataLoader.next_step, the online graph,
scenes.build_scene: the train.py node slice, stride 0, n_frames = len(batch),
validation pairing), skipping batches with fewer than two pedestrians
(train.py:86-90); a dataset whose walk ends starts over.

Data: the CSVs under --data_root (load_traj.DATA_DIRS) or, without one, the
reference's own data files committed as fixtures (tests/golden/data_*.npz:
raw CSV arrays of eth/hotel, ucy/zara01, ucy/zara02, ucy/univ).
"""
from __future__ import annotations

import os
from types import SimpleNamespace

import numpy as np

from . import networkx_graph as nxg
from .load_traj import DataLoader
from .scenes import build_scene, pack
from .synthetic import SceneBatch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURES = os.path.join(ROOT, "tests", "golden")
DATASETS = {"eth_hotel": 0, "zara01": 2, "zara02": 3, "ucy_univ": 4}   # load_traj.DATA_DIRS index
ARGS = SimpleNamespace(batch_size=16, seq_length=12, pred_len=12, obs_len=8)


def _loader(name, data_root=None):
    if data_root:
        return DataLoader(ARGS, datasets=[0, 1, 2, 3, 4, 5], start=DATASETS[name], sel=0,
                          data_root=data_root)
    return DataLoader(ARGS, raw_data=np.load(os.path.join(FIXTURES, f"data_{name}.npz"))["raw_data"])


def _walk(name, data_root=None, min_peds=2):
    """Endless scene stream of one dataset (train.py's batch walk, restarted
    at the end of the data)."""
    loader = _loader(name, data_root)
    while True:
        loader.reset_data_pointer()
        graph = nxg.online_graph(ARGS)
        frame, got = 1, 0
        for _ in range(loader.num_batches):
            batch, tgt, _ = loader.next_step()
            if len(batch) == 0:
                break
            g = graph.ConstructGraph(current_batch=batch, framenum=int(frame), future_traj=tgt)
            sc = build_scene(batch, tgt, g, loader, frame)
            for k in batch:
                frame = k
            if sc.window.shape[1] >= min_peds:
                got += 1
                yield sc
        if got == 0:
            raise ValueError(f"{name}: no batch with >= {min_peds} pedestrians")


def real_scenes(S, names=tuple(DATASETS), data_root=None):
    walks = [_walk(n, data_root) for n in names]
    return [next(walks[i % len(walks)]) for i in range(S)]


def real_batch(S, H, names=tuple(DATASETS), data_root=None, nmax=None, seed=1) -> SceneBatch:
    """S real scenes as one launch's inputs (numpy, float32): stride 0,
    per-scene n_frames and ped_mask, G ~ N(0, 1) (ctxt.png absent, quirk Q7),
    h0 = 0 (chain cut)."""
    pk = pack(real_scenes(S, names, data_root), H, nmax=nmax)
    rng = np.random.default_rng(seed)
    return SceneBatch(pos=pk["pos"], vislet=pk["vislet"],
                      G=rng.standard_normal((S, 16, 8)).astype(np.float32),
                      targets=pk["targets"], n_active=pk["n_active"],
                      h0=np.zeros((S, 16, H), np.float32), stride=0,
                      n_frames=pk["n_frames"], ped_mask=pk["ped_mask"])
