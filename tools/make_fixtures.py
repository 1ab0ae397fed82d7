#!/usr/bin/env python3
"""Generate golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container, where /root/reference exists (no-op
elsewhere).  It imports the reference's own data-side modules
(load_traj.py, networkx_graph.py, argParser.py — numpy/networkx/torch only)
and records their outputs for the first batches of each dataset:

  * DataLoader.load_dataset (load_traj.py:114-150) on the dataset CSV,
  * the frame dict the reference READS: DataLoader.__init__ loads
    trajectories_0.cpkl whenever it exists (load_traj.py:95-112); each shipped
    pickle holds frame_preprocess (load_traj.py:234-256) over the WHOLE CSV.
    The dict is restated here over the whole CSV and checked against the
    pickle WITHOUT unpickling it: ``pickle.dumps(dict, protocol=2)`` (as the
    reference wrote it, :254-256, with numpy 1.x's module name and dtype
    arguments) must equal the file's bytes.  The file's sha256 is recorded.
    eth/univ ships no pickle: the reference builds the dict over the split
    (:97-99), and so does the fixture,
  * DataLoader.next_step (load_traj.py:153-224) — batches and targets,
  * online_graph.ConstructGraph + get_node_attr (networkx_graph.py:30-73,
    114-150) as called by train.py:74-90 / 280-299 (float frame key cast to
    int, quirk Q9) and by sample.py:150-164 (fresh graph, framenum 0),
  * the batch_v preprocessing of train.py:76-85 and sample.py:152-164.

Writes tests/golden/data_<name>.npz (inputs and expected outputs; data only).

Also decodes the TF tensor-bundle checkpoint
save/g2k_mcrAttn_model_kfold_train_4_0.ckpt-79 (.index SSTable of
BundleEntryProto + raw .data) and stores, for every model copy, weight_c,
cost and the forward Variable holding weight_c @ cost (models/g2k_lstm_mcr.py:122)
as tests/golden/ckpt_mcr_attn.npz — a known-answer test for the oracle —
and the GridLSTMCell weights of save/g2k_mcr_model_val_0.ckpt-0 as
tests/golden/ckpt_gridlstm.npz.
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
OUT = os.path.join(ROOT, "tests", "golden")

DATASETS = {  # name -> (dir relative to data/, csv selection index 0)
    "eth_hotel": "eth/hotel/",
    "eth_univ": "eth/univ/",
    "zara01": "ucy/zara/zara01/",
    "zara02": "ucy/zara/zara02/",
    "ucy_univ": "ucy/univ/",
}
N_BATCHES = 3


def frame_dict_from_csv(dl, whole):
    """load_traj.py:234-256 restated (the reference writes it to a pickle) over
    the whole CSV (``whole``: what the shipped pickles hold) or over the split
    the loader holds (frameList / pedsPerFrameList, when no pickle exists)."""
    cols = dl.raw_data if whole else dl.pedsPerFrameList
    frames = cols[0]
    frame_data = {i: {} for i in frames}
    ppfl = np.transpose(cols[0:4])
    fp = dl.frame_pointer
    while fp <= max(frames):
        frame_data[fp] = [{ped: [px, py]} for (ind, ped, px, py) in ppfl if ind == fp]
        fp += dl.diff
    return frame_data


def pickle_numpy1(frame_data):
    """pickle.dump(frame_data, f, protocol=2) (load_traj.py:254-256) as numpy 1.x
    writes it: numpy >= 2 names the scalar reducer numpy._core.multiarray and
    passes the dtype's align/copy flags as bools (NEWFALSE/NEWTRUE) where
    numpy 1.x wrote numpy.core.multiarray and the ints 0 / 1."""
    import pickle
    b = pickle.dumps(frame_data, protocol=2)
    b = b.replace(b"cnumpy._core.multiarray\nscalar\n", b"cnumpy.core.multiarray\nscalar\n")
    return b.replace(b"X\x02\x00\x00\x00f8q\x03\x89\x88\x87",
                     b"X\x02\x00\x00\x00f8q\x03K\x00K\x01\x87", 1)


def pickled_dict_check(d, frame_data):
    """-> (mode, sha256 of trajectories_0.cpkl or ""): the pickle's bytes
    must equal the restated whole-CSV dict's (never unpickled: a byte
    comparison of the file with our own pickle.dumps output)."""
    import hashlib
    pk = os.path.join(d, "trajectories_0.cpkl")
    if not os.path.exists(pk):
        return "split", ""
    raw = open(pk, "rb").read()
    if pickle_numpy1(frame_data) != raw:
        raise AssertionError(f"{pk}: bytes differ from the whole-CSV frame dict")
    return "whole", hashlib.sha256(raw).hexdigest()


def ref_loader(rel):
    """The reference's DataLoader on data/<rel> (built with __new__: its
    __init__ hard-codes /home/siri0005/..., quirk Q8), its own load_dataset,
    and the frame dict it would read, restated from the CSV (whole CSV when
    trajectories_0.cpkl exists, checked against the file's bytes)."""
    sys.path.insert(0, REF)
    import argParser
    import load_traj

    args = argParser.ArgsParser().parser.parse_args([])
    d = os.path.join(REF, "data", rel)
    csv = sorted(glob.glob(d + "*.csv"))[0]
    dl = load_traj.DataLoader.__new__(load_traj.DataLoader)
    dl.batch_size, dl.seq_length = args.batch_size, args.seq_length
    dl.pred_len, dl.obs_len, dl.diff = args.pred_len, args.obs_len, args.obs_len
    dl.infer = False
    dl.current_dir = d
    dl.load_dataset(csv)
    whole = os.path.exists(os.path.join(d, "trajectories_0.cpkl"))
    dl.trajectories = frame_dict_from_csv(dl, whole)
    dl.dict_mode, dl.pickle_sha256 = pickled_dict_check(d, dl.trajectories) if whole else ("split", "")
    dl.num_batches = int((len(dl.frameList) / dl.seq_length) / dl.batch_size)
    return dl, args


def _pack(prefix, recs, out):
    """Per-batch records -> flat arrays: scalars stacked, arrays concatenated
    along axis 0 with a <field>_off offsets array, digests as strings."""
    fields = []
    for r in recs:
        fields += [f for f in r if f not in fields]
    out[prefix + "count"] = np.int64(len(recs))
    for f in fields:
        vals = [r.get(f) for r in recs]
        if all(isinstance(v, str) or v is None for v in vals):
            out[prefix + f] = np.array(["" if v is None else v for v in vals])
        elif all(v is None or np.ndim(v) == 0 for v in vals):
            out[prefix + f] = np.array([np.nan if v is None else v for v in vals], dtype=np.float64)
        else:
            arrs = [np.asarray(v) for v in vals if v is not None]
            tail = arrs[0].shape[1:]
            arrs = [np.zeros((0,) + tail) if v is None else np.asarray(v).reshape((-1,) + tail)
                    for v in vals]
            out[prefix + f] = np.concatenate(arrs, axis=0)
            out[prefix + f + "_off"] = np.cumsum([0] + [len(a) for a in arrs]).astype(np.int64)


SAMPLE_OFFSETS = (0, 5, 11)      # sample walks from seed + 8k (k = 0: sample.py itself)
TRAIN_EPOCHS = 3


def make_walk_fixture(name, rel):
    """Full walks of the reference's data side over EVERY batch
    (tools/ref_walks.py): the train.py training walk (3 epochs), the
    validation walk from the data seed (--valid_from_seed) and from 0 (the
    reference's own reset: no batch), and sample.py's walk from the seed and
    from two shifted pointers.  Writes tests/golden/walk_<name>.npz."""
    out = {}
    dl, args = ref_loader(rel)
    import networkx_graph
    import ref_walks

    recs, events = ref_walks.train_walk(dl, networkx_graph, args, TRAIN_EPOCHS)
    _pack("tw_", recs, out)
    out["tw_events"] = np.array([f"{ev[0]}:{ev[1]}" + (f":{ev[2]}" if len(ev) > 2 else "")
                                 for ev in events])
    for tag, start in (("vs_", dl.seed), ("v0_", 0)):
        dl, args = ref_loader(rel)
        recs, info = ref_walks.valid_walk(dl, networkx_graph, args, start)
        _pack(tag, recs, out)
        out[tag + "end"] = np.array(info["end"])
        out[tag + "valid_num_batches"] = np.int64(info["valid_num_batches"])
        out[tag + "valid_frame_pointer"] = np.int64(info["valid_frame_pointer"])
    for k in SAMPLE_OFFSETS:
        dl, args = ref_loader(rel)
        recs = ref_walks.sample_walk(dl, networkx_graph, args, offset=k)
        if k:                 # shifted walks: keys, counts and digests only
            recs = [dict(b=r["b"], fp=r["fp"], keys=r["keys"], P=r["P"],
                         npl_digest=ref_walks.digest(r["node_ids"], r["npl"]),
                         tgt_digest=ref_walks.digest(r["node_tlens"], r["node_targets"]))
                    for r in recs]
        _pack(f"s{k}_", recs, out)
    np.savez_compressed(os.path.join(OUT, f"walk_{name}.npz"), **out)
    return {k: v.shape for k, v in out.items() if k.endswith("count")}


def make_data_fixture(name, rel):
    sys.path.insert(0, REF)
    import argParser
    import load_traj
    import networkx_graph

    args = argParser.ArgsParser().parser.parse_args([])
    d = os.path.join(REF, "data", rel)
    csv = sorted(glob.glob(d + "*.csv"))[0]
    dl = load_traj.DataLoader.__new__(load_traj.DataLoader)
    dl.batch_size, dl.seq_length = args.batch_size, args.seq_length
    dl.pred_len, dl.obs_len, dl.diff = args.pred_len, args.obs_len, args.obs_len
    dl.infer = False
    dl.current_dir = d
    dl.load_dataset(csv)
    whole = os.path.exists(os.path.join(d, "trajectories_0.cpkl"))
    dl.trajectories = frame_dict_from_csv(dl, whole)
    mode, sha = pickled_dict_check(d, dl.trajectories) if whole else ("split", "")
    dl.num_batches = int((len(dl.frameList) / dl.seq_length) / dl.batch_size)
    dl.reset_data_pointer()
    graph = networkx_graph.online_graph(args)

    # next_step's `targets={}` default is one dict shared by every call in the
    # process (load_traj.py:153): start each dataset's fixture from empty
    load_traj.DataLoader.next_step.__defaults__[0].clear()
    rec = {"raw_data": dl.raw_data, "num_batches": np.int64(dl.num_batches),
           "frame_dict": np.array(mode), "pickle_sha256": np.array(sha),
           "dict_keys": np.int64(len(dl.trajectories))}
    frame = 1                                  # train.py:34
    for b in range(N_BATCHES):
        batch, target_traj, fptr = dl.next_step()
        keys = np.array(list(batch.keys()), dtype=np.float64)
        # the frame dicts of this batch, flattened: (frame key, ped id, x, y)
        flat = [(k, float(ped), pos[0], pos[1]) for k in batch for item in batch[k]
                for ped, pos in item.items()]
        rec[f"b{b}_keys"] = keys
        rec[f"b{b}_frames_flat"] = np.array(flat, dtype=np.float64).reshape(-1, 4)
        rec[f"b{b}_frame_pointer"] = np.float64(fptr)
        tkeys = list(target_traj.keys())
        rec[f"b{b}_target_ids"] = np.array(tkeys, dtype=np.int64)
        rec[f"b{b}_target_lens"] = np.array([len(target_traj[k]) for k in tkeys], dtype=np.int64)
        rec[f"b{b}_target_flat"] = (np.concatenate([np.asarray(target_traj[k], dtype=np.float64)
                                                    for k in tkeys]).reshape(-1, 2)
                                    if tkeys else np.zeros((0, 2)))
        # train.py path (stateful graph; framenum = previous frame key, cast to int: Q9)
        g = graph.ConstructGraph(current_batch=batch, framenum=int(frame), future_traj=target_traj)
        npl = g.get_node_attr(param="node_pos_list")
        rec[f"b{b}_node_ids"] = np.array(list(npl.keys()), dtype=np.int64)
        rec[f"b{b}_node_pos_list"] = np.array(list(npl.values()), dtype=np.float64).reshape(-1, 8, 2)
        bv = np.array(list(npl.values()))
        if len(bv.shape) > 1:
            bv = np.linalg.norm(np.array(bv)[int(frame):int(frame) + args.obs_len], axis=2).squeeze()
            bv = np.transpose(bv)
        rec[f"b{b}_batch_v_train"] = np.asarray(bv, dtype=np.float64)
        rec[f"b{b}_framenum"] = np.int64(int(frame))
        # sample.py path: fresh graph each batch, framenum 0, time slice
        gs = networkx_graph.online_graph(args).ConstructGraph(current_batch=batch, framenum=0,
                                                              future_traj=target_traj)
        npl_s = np.array(list(gs.get_node_attr(param="node_pos_list").values()))
        bvs = np.transpose(np.linalg.norm(npl_s[:, 0:args.obs_len], axis=2))
        rec[f"b{b}_batch_v_sample"] = bvs.astype(np.float64)
        tg = gs.get_node_attr(param="targets")
        rec[f"b{b}_sample_target_ids"] = np.array(list(tg.keys()), dtype=np.int64)
        rec[f"b{b}_sample_target_lens"] = np.array([len(v[0]) for v in tg.values()], dtype=np.int64)
        rec[f"b{b}_sample_targets_flat"] = (np.concatenate([np.asarray(v[0], dtype=np.float64).reshape(-1, 2)
                                                             for v in tg.values()])
                                            if tg else np.zeros((0, 2)))
        for k in batch:                        # train.py:197 leaves `frame` at the last key
            frame = k
    np.savez_compressed(os.path.join(OUT, f"data_{name}.npz"), **rec)
    return rec


# TF tensor bundle reader: the package's (multimodaltraj_2_amd/checkpoint.py)
sys.path.insert(0, ROOT)
from multimodaltraj_2_amd.checkpoint import read_bundle  # noqa: E402


def make_ckpt_fixture():
    """Known answers from the reference's own checkpoints.

    mcrAttn: the forward Variable [24, 8] created at models/g2k_lstm_mcr.py:122
    equals weight_c @ (the forward cost Variable [8, 8] of :112) for the
    model copies whose variables were initialised in one run (5 of 20).
    mc: g2k_lstm_mc's forward Variables [24, 8] / [24, 304] are all zero
    (cost = d placeholder / d Variable = 0, models/g2k_lstm_mc.py:59-66)."""
    t = read_bundle(os.path.join(REF, "save", "g2k_mcrAttn_model_kfold_train_4_0.ckpt-79"))
    out = {}
    wcs = {k: v for k, v in sorted(t.items()) if k.endswith("/weight_c")}
    c88 = {k: v for k, v in t.items() if k.startswith("Variable") and v.shape == (8, 8)}
    fwd = {k: v for k, v in t.items() if k.startswith("Variable") and v.shape == (24, 8)}
    n = 0
    for gk, wc in wcs.items():
        for ck, c in c88.items():
            prod = wc @ c
            for k, v in fwd.items():
                if np.abs(v - prod).max() <= 1e-15 * max(1.0, np.abs(v).max()):
                    out[f"pair{n}_weight_c"], out[f"pair{n}_cost"], out[f"pair{n}_temp"] = wc, c, v
                    out[f"pair{n}_names"] = np.array([gk, ck, k])
                    n += 1
    out["n_pairs"] = np.int64(n)
    tm = read_bundle(os.path.join(REF, "save", "g2k_mc_model_kfold_train_4_0.ckpt-79"))
    g = sorted(k for k in tm if k.endswith("/weight_c"))[0].rsplit("/", 1)[0]
    out["mc_weight_c"] = tm[g + "/weight_c"]
    out["mc_weight_o"] = tm[g + "/weight_o"]
    zeros = [k for k, v in tm.items() if k.startswith("Variable") and v.shape in ((24, 8), (24, 304))]
    out["mc_forward_all_zero"] = np.array([bool(np.all(tm[k] == 0)) for k in zeros])
    np.savez_compressed(os.path.join(OUT, "ckpt_mcr_attn.npz"), **out)
    return n, len(t)


def make_ckpt_scope_fixture(k=289, group=1):
    """One model copy of the reference's mcrAttn checkpoint under its own
    variable names (krnl_weights_<k>/*, krnl_embed_<k>/weight_r,
    weight_input_<k>/*) plus the forward Variables of the group whose
    weight_c @ cost matches (Variable_<1728+6g> .. +5), re-encoded as a small
    TF bundle: the fixture for checkpoint.load_params and the D = 10 model
    tests."""
    from multimodaltraj_2_amd.checkpoint import write_bundle
    t = read_bundle(os.path.join(REF, "save", "g2k_mcrAttn_model_kfold_train_4_0.ckpt-79"))
    keep = {n: v for n, v in t.items()
            if n.split("/")[0] in (f"krnl_weights_{k}", f"krnl_embed_{k}", f"weight_input_{k}")}
    base = 1728 + 6 * group
    keep.update({f"Variable_{base + i}": t[f"Variable_{base + i}"] for i in range(6)})
    write_bundle(os.path.join(OUT, f"ckpt_mcrattn_{k}"), keep)
    return sorted(keep)


def make_attn_range_fixture():
    """A second known answer from the reference's checkpoint: in every model
    copy (20) of save/g2k_mcrAttn_model_kfold_train_4_0.ckpt-79 the forward's
    Variables are created in the order of models/g2k_lstm_mcr.py:102-122 —
    ngh = Variable(lambda * ngh) [10, 8] (:102), then
    attn = Variable(ngh @ (E * Rm)) [10, 10] (:105-106) — six Variables per
    copy from Variable_1728.  Whatever E * Rm was (its placeholder defaults are
    re-drawn per evaluation), the saved attn lies in the column space of the
    saved ngh: attn = ngh @ M with M = pinv(ngh) @ attn.  Stores the pairs and
    the relative residuals |attn - ngh pinv(ngh) attn| / |attn|, and for the
    record the relations that do NOT hold (the E-like [8, 10] Variable is no
    factor: cost != E @ ngh, attn != ngh @ E)."""
    t = read_bundle(os.path.join(REF, "save", "g2k_mcrAttn_model_kfold_train_4_0.ckpt-79"))
    out, res, bad_cost, bad_attn = {}, [], [], []
    for gi in range(20):
        base = 1728 + 6 * gi
        g, A, E, C = (t[f"Variable_{base + i}"] for i in range(4))
        assert g.shape == (10, 8) and A.shape == (10, 10) and E.shape == (8, 10) and C.shape == (8, 8)
        out[f"ngh{gi}"], out[f"attn{gi}"] = g, A
        M = np.linalg.lstsq(g, A, rcond=None)[0]
        res.append(np.abs(A - g @ M).max() / np.abs(A).max())
        bad_cost.append(np.abs(E @ g - C).max() / np.abs(C).max())
        bad_attn.append(np.abs(g @ E - A).max() / np.abs(A).max())
    out["names"] = np.array([f"Variable_{1728 + 6 * gi}/Variable_{1729 + 6 * gi}" for gi in range(20)])
    out["residual"] = np.array(res)
    out["cost_vs_E_ngh"] = np.array(bad_cost)
    out["attn_vs_ngh_E"] = np.array(bad_attn)
    np.savez_compressed(os.path.join(OUT, "ckpt_attn_range.npz"), **out)
    return max(res), min(bad_cost), min(bad_attn)


def make_gridlstm_fixture():
    """GridLSTMCell weights (helper.py:31-39) from the reference's own
    checkpoint save/g2k_mcr_model_val_0.ckpt-0: W_f_0_0 [8,6], B_f_0 [6] and
    the four peephole diagonals [2] — realistic weights for the a6 kernel's
    tests (its outputs stay unpinned: no reference run exists)."""
    t = read_bundle(os.path.join(REF, "save", "g2k_mcr_model_val_0.ckpt-0"))
    out, names = {}, []
    for key, suf in (("W", "W_f_0_0"), ("b", "B_f_0"), ("wIf", "W_I_diag_freqf_0"),
                     ("wIt", "W_I_diag_freqt_0"), ("wOf", "W_O_diag_freqf_0"),
                     ("wOt", "W_O_diag_freqt_0")):
        ks = sorted(k for k in t if k.endswith(suf))
        names.append(ks[0])
        out[key] = t[ks[0]]
    out["names"] = np.array(names)
    np.savez_compressed(os.path.join(OUT, "ckpt_gridlstm.npz"), **out)
    return names


def main():
    if not os.path.isdir(REF):
        print("no /root/reference here: fixtures are committed, nothing to do")
        return
    os.makedirs(OUT, exist_ok=True)
    if "--ckpt-only" in sys.argv:
        print("attn in range(ngh): max residual, min cost / attn mismatch:", make_attn_range_fixture())
        return
    for name, rel in DATASETS.items():
        rec = make_data_fixture(name, rel)
        print(name, {k: np.shape(v) for k, v in rec.items() if k.startswith("b0")})
        make_walk_fixture(name, rel)
    print("checkpoint pairs (weight_c @ cost == stored Variable):", make_ckpt_fixture())
    print("gridlstm weights:", make_gridlstm_fixture())
    print("mcrAttn model copy:", make_ckpt_scope_fixture())
    print("attn in range(ngh): max residual, min cost / attn mismatch:", make_attn_range_fixture())


if __name__ == "__main__":
    main()
