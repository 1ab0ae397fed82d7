"""GPU: sample.py at the reference geometry (D = num_freq_blocks = 10,
sample.py:137-332) on the committed data fixtures, with weights restored from
a copy of the reference's own checkpoint (tests/golden/ckpt_mcrattn_289: model
copy 289 of save/g2k_mcrAttn_model_kfold_train_4_0.ckpt-79, D = 10), vs the
float64 oracle (GridLSTM cell, g2k_lstm_mcr forward, get_mean_error) fed the
same draws.  Tolerance |d| <= 1e-4 * max(1, |ref|)."""
import os
import shutil

import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import checkpoint as ck
from multimodaltraj_2_amd import helper
from multimodaltraj_2_amd import sample
from multimodaltraj_2_amd.argParser import ArgsParser
from multimodaltraj_2_amd.load_traj import DataLoader
from oracle import g2k_ref as ref
from tests.conftest import close

pytestmark = pytest.mark.gpu
TOL = 1e-4
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _args(save_dir):
    a = ArgsParser().parser.parse_args([])
    a.batch_size, a.seq_length, a.pred_len, a.obs_len = 16, 12, 12, 8
    a.obs_length, a.save_dir = 8, save_dir
    return a


def _save_dir(tmp_path):
    d = tmp_path / "save"
    d.mkdir()
    for ext in (".index", ".data-00000-of-00001"):
        shutil.copy(os.path.join(GOLDEN, "ckpt_mcrattn_289" + ext), d / ("g2k_mcrAttn.ckpt-79" + ext))
    ck.write_state(str(d), str(d / "g2k_mcrAttn.ckpt-79"))
    return str(d)


@pytest.mark.parametrize("name", ["zara01", "ucy_univ"])
def test_sample_d10_restored_matches_oracle(gpu, tmp_path, name):
    args = _args(_save_dir(tmp_path))
    z = np.load(os.path.join(GOLDEN, f"data_{name}.npz"))
    dl = DataLoader(args, raw_data=z["raw_data"])
    dl.reset_data_pointer()
    restored = sample.restore_weights(args.save_dir, gpu)
    assert restored is not None and tuple(restored.Wv.shape) == (8, 12)
    D, lam, seed = args.num_freq_blocks, args.lambda_param, args.seed
    past_g, past_o = 1.0, 1.0
    done = 0
    for b, sc, _ in sample.batches(args, dl):
        ade, fde, vis_emb, pred = sample.sample_batch(args, sc, past_g, restored, gpu, seed)
        torch.cuda.synchronize()
        past_g = vis_emb
        # the oracle, fed the same draws (float32 values, float64 arithmetic)
        n = sc.window.shape[1]
        rng = np.random.default_rng(seed)
        Wi = rng.standard_normal((n, D)).astype(np.float32).astype(np.float64)
        Wii = rng.standard_normal((D, 8)).astype(np.float32).astype(np.float64)
        bv_ = np.linalg.norm(sc.window.astype(np.float32), axis=2).astype(np.float64)
        inputs = Wii @ (bv_ @ Wi)
        vemb = sc.vislet[:, :n].astype(np.float32) @ Wi
        cell = helper.GridLSTMCell(num_units=args.num_layers, feature_size=args.grid_size,
                                   frequency_skip=args.grid_size, use_peepholes=True,
                                   num_frequency_blocks=[D // args.grid_size], seed=seed, device=gpu)
        ng, _ = ref.gridlstm_cell(inputs[:, :8], np.zeros((D, args.rnn_size)), cell.W.cpu().numpy(),
                                  cell.b.cpu().numpy(), tuple(cell.peep.cpu().numpy()))
        w = {k: v.cpu().numpy() for k, v in sample.model_weights(restored, n, D, 8, seed + 1, gpu).items()}
        assert np.array_equal(w["weight_v"], ck.read_bundle(os.path.join(GOLDEN, "ckpt_mcrattn_289"))
                              ["krnl_weights_289/weight_v"].astype(np.float32))
        o = ref.mcr_forward(np.concatenate([inputs, vemb], 0), past_o * vemb, lam * ng, w["weight_v"],
                            w["bias_v"], w["weight_r"], w["weight_c"], w["weight_o"], lam)
        past_o = vemb
        assert close(pred.cpu().numpy(), o["pred_path_band"]) <= TOL
        e_ade, e_fde, _ = ref.get_mean_error(np.transpose(o["pred_path_band"], (2, 1, 0)), sc.targets, 8, n)
        assert abs(ade - e_ade) <= TOL * max(1.0, abs(e_ade))
        assert abs(fde - e_fde) <= TOL * max(1.0, abs(e_fde))
        done += 1
        if done == 3:
            break
    assert done >= 1


def test_sample_run_timings_and_results_pickle(gpu, tmp_path):
    """sample.py:256-348: every batch prints the per-stage wall times (hipEvent
    timers here) and the run pickles results = [(x_batch, complete_traj,
    obs_length)] with complete_traj = pred_path_band transposed (2, 1, 0)
    (sample.py:326, 340, 346-348)."""
    import pickle
    args = _args(_save_dir(tmp_path))
    z = np.load(os.path.join(GOLDEN, "data_zara01.npz"))
    dl = DataLoader(args, raw_data=z["raw_data"])
    dl.reset_data_pointer()
    dl.num_batches = 3
    lines = []
    total, final, results = sample.run(args, dl, gpu, log=lambda *a: lines.append(" ".join(map(str, a))))
    assert len(results) == len(total) >= 1
    path = sample.save_results(results, args.save_dir, log=lines.append)
    assert path == os.path.join(args.save_dir, "social_results.pkl")
    with open(path, "rb") as f:          # our own file
        back = pickle.load(f)
    # the same batches again: pred per batch, to compare with the pickle
    dl2 = DataLoader(args, raw_data=z["raw_data"])
    dl2.reset_data_pointer()
    dl2.num_batches = 3
    restored = sample.restore_weights(args.save_dir, gpu)
    past = 1.0
    for (xb, ct, obs), (b, sc, x_batch) in zip(back, sample.batches(args, dl2)):
        _, _, past, pred = sample.sample_batch(args, sc, past, restored, gpu, args.seed)
        assert obs == 8 and list(xb.keys()) == list(x_batch.keys())
        np.testing.assert_array_equal(ct, np.transpose(pred.cpu().numpy(), (2, 1, 0)))
        assert ct.shape == (sc.window.shape[1], 12, 2)
    for key in ("social mask grid", "static mask grid", "combined mask grid", "predictive kernel",
                "Relational inference calculation took", "Multi-Cued model (MCR) sampling time"):
        got = [float(l.split("= ")[1].split()[0]) for l in lines if key in l]
        assert len(got) == len(results) and all(v >= 0 for v in got), key
    assert sum(1 for l in lines if "SAMPLING A NEW TRAJECTORY" in l) == len(results)
