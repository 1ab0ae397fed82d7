"""Real-data scene plans on the host (no GPU): distinct scenes, every dataset,
the native planner against the Python walk (sample.py's scene per frame
pointer: load_traj.next_step + a fresh online graph at framenum 0, time slice),
and the host expansion of the plans."""
import os

import numpy as np
import pytest

from multimodaltraj_2_amd import realdata as rd
from multimodaltraj_2_amd import walks

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
RAW = {n: np.load(os.path.join(GOLDEN, f"data_{n}.npz"))["raw_data"] for n in rd.DATASETS}


def _distinct_rows(a):
    a = np.ascontiguousarray(a.reshape(len(a), -1))
    return len(np.unique(a.view(np.dtype((np.void, a.shape[1] * a.itemsize)))))


@pytest.mark.parametrize("S", [128, 1024])
def test_plans_are_distinct_scenes(S):
    p = rd.plan_scenes(S, RAW)
    assert p.S == S
    assert set(p.names) == set(rd.DATASETS)
    assert (p.n_active >= 2).all() and (p.n_active <= p.Nmax).all()
    assert len(set(zip(p.names, p.pointers))) == S                       # distinct windows
    rows = np.concatenate([p.pos_col.reshape(S, -1), p.tgt_col.reshape(S, -1)], axis=1)
    assert _distinct_rows(rows) == S                                     # distinct contents
    h = p.host(F=2)
    assert _distinct_rows(np.concatenate([h["pos"].reshape(S, -1),
                                          h["targets"][:, 0].reshape(S, -1)], axis=1)) == S
    assert len(set(p.n_frames.tolist())) > 1                             # ragged frame loops


def test_fold_datasets():
    assert rd.fold_datasets(4) == ["eth_hotel", "zara01", "zara02"]
    assert rd.fold_datasets(2) == ["eth_hotel", "zara02", "ucy_univ"]
    p = rd.plan_scenes(64, {n: RAW[n] for n in rd.fold_datasets(4)})
    assert "ucy_univ" not in p.names and p.Nmax == 32


@pytest.mark.parametrize("name", list(rd.DATASETS))
def test_plan_matches_python_walk(name):
    """Every scene of a dataset's plan (first 40 pointers) equals what the
    Python walk builds from the same pointer: window (time slice of the fresh
    graph), node targets, frame count."""
    src = rd.SceneSource(name, RAW[name])
    plan = src.plan(40)
    xy = src.xy.astype(np.float64)
    dl = src.loader
    for j in range(40):
        rec = _one(dl, src.pointers[j])
        P = len(rec.node_ids)
        assert int(plan["n_nodes"][j]) == P
        assert int(plan["n_keys"][j]) == rec.n_frames
        if P == 0:
            continue
        pc = plan["pos_col"][j][:, :P]
        got = np.where(pc[..., None] >= 0, xy[np.maximum(pc, 0)], 0)
        np.testing.assert_array_equal(got.astype(np.float32),
                                      rec.window.astype(np.float32))
        tc = plan["tgt_col"][j][:P]
        tv = np.where(tc[..., None] >= 0, xy[np.maximum(tc, 0)], 0)
        want = np.zeros((P, 12, 2))
        for i, t in enumerate(rec.extra["node_targets"]):
            t = np.asarray(t, np.float64).reshape(-1, 2)[:12]
            want[i, :len(t)] = t
        np.testing.assert_array_equal(tv.astype(np.float32), want.astype(np.float32))


def _one(dl, fp):
    """sample_walk's first record from frame pointer fp (= seed + 8 m)."""
    m = int(round((fp - dl.seed) / dl.diff))
    return next(walks.sample_walk(dl, rd.ARGS, offset=m, max_batches=1))
