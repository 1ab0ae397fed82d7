"""GPU: train.py's two legs through the entry point (multimodaltraj_2_amd/train.py)
on the reference's data files (tests/golden/data_*.npz written as a data root)
vs the float64 oracle run batch by batch over the same walk.

Training leg: every batch of every epoch of the fold's first dataset (the
reference's e / frame / counters are set once per left-out dataset,
train.py:29-36), in one launch per epoch, the hidden state chained batch after
batch: the raw-vector logs (train.py:254-276, 346-351) == oracle.train_log_errors
on the oracle's predictions, the chained h == the oracle's sequential chain, the
counts file == the reference replay's counters (tests/golden/walk_*.npz).
Validation leg: fresh graph, frame = 1 (train.py:374, 392); per-batch ADE / FDE
== oracle.batch_metrics; train() end to end validates the same way.
Tolerance 1e-4 * max(1, |ref|); h: close_h."""
import os
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd import train as tr
from multimodaltraj_2_amd import walks
from multimodaltraj_2_amd.argParser import ArgsParser
from multimodaltraj_2_amd.load_traj import DataLoader
from multimodaltraj_2_amd.scenes import pack, scene_from_record
from oracle import g2k_ref as ref
from tests.conftest import close, close_h

pytestmark = pytest.mark.gpu
TOL = 1e-4
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FIRST = {3: ("zara01", 2), 2: ("zara02", 3)}       # leaveDataset -> the fold's first dataset


def _args(tmp_path, data_root, leave, epochs=3):
    a = ArgsParser().parser.parse_args([])
    a.num_epochs, a.log_dir, a.save_dir, a.leaveDataset = epochs, str(tmp_path), "", leave
    a.data_root = data_root
    return a


def _oracle_record(args, loader, rec, pairing, h0, encoder=None):
    sc = scene_from_record(rec, loader, pairing=pairing)
    pk = pack([sc], args.rnn_size, nmax=tr.NODE_SLICE_NMAX)
    w = fs.init_params(tr.NODE_SLICE_NMAX, seed=args.seed).numpy()
    G = tr.context_G(args.seed)[0]
    n = int(pk["n_active"][0])
    return ref.scene_step(pk["pos"][0], pk["vislet"][0], G, w, pk["targets"][0], n, h0,
                          n_frames=int(pk["n_frames"][0]), stride=0, lam=args.lambda_param,
                          ped_mask=pk["ped_mask"][0].astype(bool), encoder=encoder)


@pytest.mark.parametrize("leave", [3, 2])
def test_training_leg_every_batch(gpu, tmp_path, data_root, leave):
    name, d = FIRST[leave]
    args = _args(tmp_path, data_root, leave)
    params = tr.leg_params(args, gpu)
    summary, h, counters = tr.training_leg(args, gpu, params, log=lambda s: None)
    # the oracle over the same walk, batch after batch, h chained
    loader = DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=d, sel=0, data_root=data_root)
    h_ref = np.zeros((16, args.rnn_size))
    euc, fde, ran = [], [], 0
    for rec in walks.train_walk(loader, args, args.num_epochs):
        if isinstance(rec, str) or rec.n < 0:
            continue
        pr, h_ref, m, _ = _oracle_record(args, loader, rec, "train_log", h_ref)
        for f in range(rec.n_frames):
            e_, d_ = ref.train_log_errors(pr[f], rec.target_traj)
            euc += e_
            fde += d_
        ran += 1
    assert ran == len(summary[d]) and ran > 3
    assert close_h(h[0].cpu().numpy(), h_ref)
    got_f = np.loadtxt(tmp_path / f"g2k_MPC_fde_log_kfold_{d}.csv", delimiter=",").reshape(-1, 2)
    got_e = np.loadtxt(tmp_path / f"g2k_MPC_error_log_kfold_{d}.csv", delimiter=",")
    assert len(fde) > 0 and got_f.shape == (len(fde), 2)
    assert close(got_f, np.array(fde)) <= TOL
    assert close(got_e, np.concatenate([np.ravel(x) for x in euc])) <= TOL
    # the counts file: the reference replay's counters after the last batch
    z = np.load(os.path.join(GOLDEN, f"walk_{name}.npz"))
    ok = z["tw_n"] >= 0
    want_t, want_e = int(z["tw_num_targets"][ok][-1]), int(z["tw_num_end_targets"][ok][-1])
    for dd in sorted({2, 3, 4} - {leave}):              # every dataset of the fold writes one
        txt = open(tmp_path / f"g2k_lstm_counts_{dd}.txt").read()
        assert txt == f"Dataset {dd}= ADE steps {want_t}\nFDE steps = {want_e}"


@pytest.mark.parametrize("name,d,leave", [("zara01", 2, 2), ("ucy_univ", 4, 5)])
def test_validation_leg_matches_oracle(gpu, tmp_path, data_root, name, d, leave):
    args = _args(tmp_path, data_root, leave)
    params = tr.leg_params(args, gpu)
    logs = []
    mk = lambda: DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=d, sel=0,  # noqa: E731
                            data_root=data_root)
    # the reference's frame pointer 0 finds no key of these files: no batch
    assert tr.validate(args, gpu, params, log=logs.append, loader=mk()) == ([], [])
    ade, fde = tr.validate(args, gpu, params, log=logs.append, loader=mk(), start_pointer=None)
    loader = mk()
    h_ref = np.zeros((16, args.rnn_size))
    want_a, want_f = [], []
    for rec in walks.valid_walk(loader, args, start_pointer=loader.seed):
        if rec.n < 0:
            break
        pr, h_ref, m, _ = _oracle_record(args, loader, rec, "row", h_ref)
        if rec.n > 0:
            a, f = ref.batch_metrics(m, leave_dataset=leave, num_nodes=rec.n)
            if np.isfinite(a):
                want_a.append(a)
                want_f.append(f)
    assert len(ade) == len(want_a) and len(ade) > 0
    assert close(ade, want_a) <= TOL and close(fde, want_f) <= TOL
    assert any("Cross-Validation total mean error (ADE)" in s for s in logs)


def test_train_entry_point_validates_on_a_fresh_graph(gpu, tmp_path, data_root):
    """train() runs the training leg, then the validation leg from frame 1 on
    a fresh graph (train.py:374, 392) — the same numbers as validate() alone."""
    args = _args(tmp_path, data_root, 2, epochs=1)
    args.valid_from_seed, args.device = 1, "cuda:0"
    logs = []
    tr.train(args, log=logs.append)
    alone = []
    tr.validate(args, gpu, tr.leg_params(args, gpu), log=alone.append, start_pointer=None)
    got = [s for s in logs if s.startswith("Cross-Validation")]
    assert got == [s for s in alone if s.startswith("Cross-Validation")] and len(got) == 2
    assert os.path.exists(tmp_path / "g2k_lstm_counts_3.txt")


def test_training_leg_with_grid_lstm_encoder(gpu, tmp_path, data_root):
    """--use_grid_lstm 1: the vis/loc encoder's GridLSTMCell in every frame
    (train.py:201-207, its output as st_embeddings, the hidden state entering
    the frame as its state): one sequential chain through every batch of the
    epoch on the GPU (encoder_step.EncoderChain) == the oracle's scene_step
    with gridlstm_cell chained in, batch after batch (h: close_h; the per-frame
    training-log vectors, which now differ frame to frame: 1e-4).  The cell is
    third-party (TF contrib): parity unpinned against TF (row a6)."""
    leave = 3
    name, d = FIRST[leave]
    args = _args(tmp_path, data_root, leave, epochs=1)
    args.use_grid_lstm = 1
    params = tr.leg_params(args, gpu)
    summary, h, _ = tr.training_leg(args, gpu, params, log=lambda s: None)
    cell = tr.encoder_cell(args, gpu)
    enc = dict(W=cell.W.cpu().numpy().astype(np.float64), b=cell.b.cpu().numpy().astype(np.float64),
               peep=tuple(cell.peep.cpu().numpy().astype(np.float64)), feature_size=cell.feature_size,
               num_units=cell.num_units)
    loader = DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=d, sel=0, data_root=data_root)
    h_ref = np.zeros((16, args.rnn_size))
    euc, fde, ran, moved = [], [], 0, 0.0
    for rec in walks.train_walk(loader, args, args.num_epochs):
        if isinstance(rec, str) or rec.n < 0:
            continue
        pr, h_ref, m, _ = _oracle_record(args, loader, rec, "train_log", h_ref, encoder=enc)
        for f in range(rec.n_frames):
            e_, d_ = ref.train_log_errors(pr[f], rec.target_traj)
            euc += e_
            fde += d_
        if rec.n_frames > 1 and pr[0].size:
            moved = max(moved, float(np.abs(pr[-1] - pr[0]).max()))
        ran += 1
    assert ran == len(summary[d]) and ran > 3
    assert moved > 0.0                       # with the encoder, predictions follow the chain
    assert close_h(h[0].cpu().numpy(), h_ref)
    got_f = np.loadtxt(tmp_path / f"g2k_MPC_fde_log_kfold_{d}.csv", delimiter=",").reshape(-1, 2)
    got_e = np.loadtxt(tmp_path / f"g2k_MPC_error_log_kfold_{d}.csv", delimiter=",")
    assert len(fde) > 0 and got_f.shape == (len(fde), 2)
    assert close(got_f, np.array(fde)) <= TOL
    assert close(got_e, np.concatenate([np.ravel(x) for x in euc])) <= TOL
