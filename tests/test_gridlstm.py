"""a6 GridLSTMCell encoders (helper.py:31-39, 131-141): the HIP kernel vs the
float64 restatement oracle.gridlstm_cell.  The op is
third-party (TF 1.x contrib, absent here, version unpinned): parity is
against the restatement of the decoded graph only, i.e. "parity unpinned"
against the reference.  One case runs on the reference's own checkpoint
weights (tests/golden/ckpt_gridlstm.npz, tools/make_fixtures.py).
Tolerance (written here): |got - ref| <= 1e-4 * max(1, |ref|)."""
import os

import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import helper
from oracle import g2k_ref as ref
from tests.conftest import close

TOL = 1e-4
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ckpt_gridlstm.npz")


def _peep(z):
    return np.stack([z["wIf"], z["wIt"], z["wOf"], z["wOt"]])


def test_checkpoint_fixture_shapes():
    z = np.load(GOLD)
    assert z["W"].shape == (8, 6) and z["b"].shape == (6,)
    assert _peep(z).shape == (4, 2)
    assert all(str(n).startswith("grid_lstm_cell/") for n in z["names"])


def test_config_guard_and_no_cpu_fallback():
    with pytest.raises(NotImplementedError):
        helper.GridLSTMCell(2, 4, 2, True, [4], device="cpu")              # frequency_skip != fs
    with pytest.raises(NotImplementedError):
        helper.GridLSTMCell(2, 4, 4, True, [4], couple_input_forget_gates=False, device="cpu")
    with pytest.raises(NotImplementedError):
        helper.GridLSTMCell(3, 4, 4, True, [4], device="cpu")
    cell = helper.GridLSTMCell(2, 4, 4, True, [4], device="cpu")
    assert tuple(cell.W.shape) == (8, 6) and tuple(cell.peep.shape) == (4, 2)
    assert cell.output_size == cell.state_size == 16
    with pytest.raises(ValueError):
        cell(torch.zeros(16, 16), torch.zeros(16, 128))                     # CPU tensors


def test_oracle_blocks_chain_through_frequency_state():
    """Block k reads block k-1's (c_freq, m_freq): two blocks at once equal
    block 0 followed by a block whose m_freq input is block 0's output."""
    rng = np.random.default_rng(0)
    W, b = rng.standard_normal((8, 6)), rng.standard_normal(6)
    x, st = rng.standard_normal((5, 8)), rng.standard_normal((5, 8))
    out, ns = ref.gridlstm_cell(x, st, W, b, None)
    o0, s0 = ref.gridlstm_cell(x[:, :4], st[:, :4], W, b, None)
    assert np.allclose(out[:, :4], o0) and np.allclose(ns[:, :4], s0)
    assert not np.allclose(out[:, 4:], ref.gridlstm_cell(x[:, 4:], st[:, 4:], W, b, None)[0])


@pytest.mark.gpu
@pytest.mark.parametrize("u,fs,K,peep,R", [(2, 4, 4, True, 16), (2, 4, 2, False, 16),
                                            (1, 2, 3, True, 37), (4, 8, 2, True, 300),
                                            (4, 2, 5, False, 1)])
def test_gridlstm_matches_oracle(gpu, u, fs, K, peep, R):
    rng = np.random.default_rng(100 * u + 10 * fs + K)
    ld = 2 * u * K + 5                                  # state pitch wider than read
    x = rng.standard_normal((R, K * fs)).astype(np.float32)
    st = rng.standard_normal((R, ld)).astype(np.float32)
    W = (0.7 * rng.standard_normal((fs + 2 * u, 3 * u))).astype(np.float32)
    b = (0.3 * rng.standard_normal(3 * u)).astype(np.float32)
    P = rng.standard_normal((4, u)).astype(np.float32) if peep else None
    t = lambda a: torch.from_numpy(a).to(gpu)           # noqa: E731
    out, ns = helper.gridlstm(t(x), t(st), t(W), t(b), None if P is None else t(P),
                              feature_size=fs, num_units=u)
    torch.cuda.synchronize()
    ro, rs = ref.gridlstm_cell(x, st, W, b, None if P is None else tuple(P), feature_size=fs,
                               num_units=u)
    assert close(out.cpu().numpy(), ro) <= TOL
    assert close(ns.cpu().numpy(), rs) <= TOL


@pytest.mark.gpu
def test_encoders_on_checkpoint_weights(gpu):
    z = np.load(GOLD)
    rng = np.random.default_rng(7)
    enc = helper.neighborhood_vis_loc_encoder(hidden_size=128, hidden_len=16, num_layers=2,
                                              grid_size=4, embedding_size=64, device=gpu)
    enc.rnn.set_weights(z["W"], z["b"], _peep(z))
    x = rng.standard_normal((16, 16)).astype(np.float32)
    h = rng.standard_normal((16, 128)).astype(np.float32)
    out, st = enc.forward(torch.from_numpy(x).to(gpu), torch.from_numpy(h).to(gpu))
    torch.cuda.synchronize()
    ro, rs = ref.gridlstm_cell(x, h, z["W"], z["b"], tuple(_peep(z)))
    assert out.shape == (16, 16) and st.shape == (16, 16)
    assert close(out.cpu().numpy(), ro) <= TOL and close(st.cpu().numpy(), rs) <= TOL
    stat = helper.neighborhood_stat_enc(None, hidden_size=128, num_layers=2, grid_size=4, dim=16,
                                        device=gpu, share_with=enc)
    xs = rng.standard_normal((16, 8)).astype(np.float32)
    o2, s2 = stat.forward(torch.from_numpy(xs).to(gpu), torch.from_numpy(h).to(gpu))
    torch.cuda.synchronize()
    r2, q2 = ref.gridlstm_cell(xs, h, z["W"], z["b"], None)
    assert o2.shape == (16, 8)
    assert close(o2.cpu().numpy(), r2) <= TOL and close(s2.cpu().numpy(), q2) <= TOL


def test_tf_block_slicing_rule():
    """tf.contrib GridLSTMCell: int((ncol - feature_size) / skip) + 1 blocks;
    sample.py's 10-column input makes 2 blocks of 4 (columns 8, 9 unread)."""
    cell = helper.GridLSTMCell(2, 4, 4, True, [2], device="cpu")
    with pytest.raises(ValueError):
        cell(torch.zeros(10, 7), torch.zeros(10, 8))
    with pytest.raises(ValueError):
        cell(torch.zeros(10, 12), torch.zeros(10, 8))
