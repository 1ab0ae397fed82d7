"""Full-walk parity of the data side (a1/a2 + the walk that feeds them) against
replays of the reference's own load_traj.py / networkx_graph.py over EVERY
batch (tests/golden/walk_*.npz, made by tools/make_fixtures.py through
tools/ref_walks.py): the train.py training walk (3 epochs), the validation
walk (from the data seed and from the reference's pointer 0), and sample.py's
walk from the seed and from two shifted pointers — through the Python walks
(multimodaltraj_2_amd/walks.py) and the native planner
(g2k_traj_sample_scenes).  Bit-exact; host code only (no GPU)."""
import glob
import hashlib
import os
from types import SimpleNamespace

import numpy as np
import pytest

from multimodaltraj_2_amd import walks
from multimodaltraj_2_amd.load_traj import DataLoader

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ARGS = SimpleNamespace(batch_size=16, seq_length=12, pred_len=12, obs_len=8)
NAMES = ["eth_hotel", "eth_univ", "zara01", "zara02", "ucy_univ"]


def digest(*arrays):
    h = hashlib.sha1()
    for a in arrays:
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


class Rec:
    """Record i of a packed walk (tools/make_fixtures.py _pack)."""

    def __init__(self, z, prefix):
        self.z, self.p = z, prefix
        self.count = int(z[prefix + "count"])

    def get(self, f, i):
        z, p = self.z, self.p
        if p + f + "_off" in z.files:
            off = z[p + f + "_off"]
            return z[p + f][off[i]:off[i + 1]]
        return z[p + f][i]


def _loader(name):
    """The loader over the frame dict the reference reads for this dataset
    (the fixture's mode: "whole" where trajectories_0.cpkl ships, else "split")."""
    z = np.load(os.path.join(GOLDEN, f"data_{name}.npz"))
    return DataLoader(ARGS, raw_data=z["raw_data"], frame_dict=str(z["frame_dict"]))


def _check_targets(r, i, tgt):
    keys = list(tgt.keys())
    np.testing.assert_array_equal(np.array(keys, np.int64), r.get("tkeys", i))
    np.testing.assert_array_equal(np.array([len(tgt[k]) for k in keys]), r.get("tlens", i))
    full = (np.concatenate([np.asarray(tgt[k], np.float64).reshape(-1, 2) for k in keys])
            if keys else np.zeros((0, 2)))
    assert digest(full) == str(r.get("tdigest", i))
    head = r.get("thead", i).reshape(-1, 12, 2)
    for j, k in enumerate(keys[:len(head)]):
        t = np.asarray(tgt[k], np.float64).reshape(-1, 2)[:12]
        np.testing.assert_array_equal(t, head[j, :len(t)])


def _check_graph(r, i, rec):
    np.testing.assert_array_equal(rec.node_ids, r.get("node_ids", i))
    assert digest(rec.node_ids, rec.npl) == str(r.get("npl_digest", i))
    assert len(rec.node_ids) == int(r.get("P", i))


@pytest.mark.parametrize("name", NAMES)
def test_train_walk_every_batch(name):
    z = np.load(os.path.join(GOLDEN, f"walk_{name}.npz"))
    r = Rec(z, "tw_")
    dl = _loader(name)
    counters = {}
    recs, ends = [], 0
    for item in walks.train_walk(dl, ARGS, epochs=3, counters=counters):
        if isinstance(item, str):
            ends += 1
            continue
        recs.append((item, dict(counters)))
    assert ends == 3
    assert len(recs) == r.count
    n_fde = 0
    for i, (rec, cnt) in enumerate(recs):
        assert rec.index == (int(r.get("e", i)), int(r.get("b", i)))
        assert rec.frame == float(r.get("frame", i))
        np.testing.assert_array_equal(np.array(list(rec.batch.keys()), np.float64), r.get("keys", i))
        _check_graph(r, i, rec)
        _check_targets(r, i, rec.target_traj)
        assert rec.n == int(r.get("n", i))
        assert rec.outcome == str(r.get("outcome", i))
        if rec.n >= 0:
            np.testing.assert_array_equal(rec.window.reshape(-1), r.get("window", i).reshape(-1))
            bv = np.linalg.norm(np.transpose(rec.window, (1, 0, 2)), axis=2).T    # train.py:79, 85
            np.testing.assert_array_equal(bv.reshape(-1), r.get("batch_v", i).reshape(-1))
            assert rec.vis_off == float(r.get("vis_off", i))
            assert rec.frame_after == float(r.get("frame_after", i))
            n_fde += rec.n_frames * sum(1 for j, _ in zip(range(1, rec.n), rec.target_traj)
                                          if j in rec.target_traj)
            assert cnt["num_targets"] == int(r.get("num_targets", i))
            assert cnt["num_end_targets"] == int(r.get("num_end_targets", i))
            assert n_fde == int(r.get("n_fde", i))
    # more than batch 0 is covered: every epoch and the later (empty-slice) batches
    assert len({rec.index[0] for rec, _ in recs}) == 3


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("tag", ["vs_", "v0_"])
def test_valid_walk_every_batch(name, tag):
    z = np.load(os.path.join(GOLDEN, f"walk_{name}.npz"))
    r = Rec(z, tag)
    dl = _loader(name)
    start = dl.seed if tag == "vs_" else 0
    gen = walks.valid_walk(dl, ARGS, start_pointer=start)
    recs = []
    while True:
        try:
            recs.append(next(gen))
        except StopIteration as stop:
            end = stop.value
            break
    assert end == str(z[tag + "end"])
    assert dl.valid_num_batches == int(z[tag + "valid_num_batches"])
    assert dl.valid_frame_pointer == int(z[tag + "valid_frame_pointer"])
    assert len(recs) == r.count
    for i, rec in enumerate(recs):
        assert rec.frame == float(r.get("frame", i)) and rec.fp == float(r.get("fp", i))
        np.testing.assert_array_equal(np.array(list(rec.batch.keys()), np.float64), r.get("keys", i))
        _check_graph(r, i, rec)
        _check_targets(r, i, rec.target_traj)
        assert rec.n == int(r.get("n", i))
        assert rec.vis_off == int(r.get("vis_off", i))
        if rec.n >= 0:
            np.testing.assert_array_equal(rec.window.reshape(-1), r.get("window", i).reshape(-1))
            assert rec.frame_after == float(r.get("frame_after", i))


def _native_values(dl, out, j, nmax):
    """Positions / targets of scene j from the native plan (column -> CSV
    values, -1 -> the zero slot)."""
    xy = np.stack([dl.dict_data[2], dl.dict_data[3]], axis=1)
    P = min(int(out["n_nodes"][j]), nmax)
    pc = out["pos_col"][j][:, :P]                     # [8, P]
    npl = np.where(pc[..., None] >= 0, xy[np.maximum(pc, 0)], 0.0).transpose(1, 0, 2)
    tc = out["tgt_col"][j][:P]                        # [P, 12]
    tl = (tc >= 0).sum(axis=1)
    tv = np.where(tc[..., None] >= 0, xy[np.maximum(tc, 0)], 0.0)
    return npl, tl, tv


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("k", [0, 5, 11])
def test_sample_walk_every_batch(name, k):
    z = np.load(os.path.join(GOLDEN, f"walk_{name}.npz"))
    r = Rec(z, f"s{k}_")
    dl = _loader(name)
    recs = list(walks.sample_walk(dl, ARGS, offset=k))
    assert len(recs) == r.count > 0
    # the native planner from the reference's own frame pointers
    fps = np.array([float(r.get("fp", i)) for i in range(r.count)])
    nmax = 128
    out = _loader(name).index.sample_scenes(fps, nmax)
    for i, rec in enumerate(recs):
        assert rec.fp == fps[i]
        if i + 1 < r.count:
            assert out["next_pointer"][i] == fps[i + 1]
        keys = np.array(list(rec.batch.keys()), np.float64)
        np.testing.assert_array_equal(keys, r.get("keys", i))
        assert int(out["n_keys"][i]) == len(keys)
        P = int(r.get("P", i))
        assert len(rec.node_ids) == P == int(out["n_nodes"][i]) <= nmax
        tl = np.array([len(t) for t in rec.extra["node_targets"]], np.int64)
        tv = np.zeros((P, 12, 2))
        for j, t in enumerate(rec.extra["node_targets"]):
            t = np.asarray(t, np.float64).reshape(-1, 2)[:12]
            tv[j, :len(t)] = t
        n_npl, n_tl, n_tv = _native_values(dl, out, i, nmax)
        np.testing.assert_array_equal(n_npl, rec.npl)
        np.testing.assert_array_equal(n_tl, tl)
        np.testing.assert_array_equal(n_tv, tv)
        if k == 0:
            np.testing.assert_array_equal(rec.node_ids, r.get("node_ids", i))
            np.testing.assert_array_equal(rec.npl.reshape(-1), r.get("npl", i).reshape(-1))
            np.testing.assert_array_equal(tl, r.get("node_tlens", i))
            np.testing.assert_array_equal(tv.reshape(-1), r.get("node_targets", i).reshape(-1))
        else:
            assert digest(rec.node_ids, rec.npl) == str(r.get("npl_digest", i))
            assert digest(tl, tv) == str(r.get("tgt_digest", i))
