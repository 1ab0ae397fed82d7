"""Known answers of the model half from the reference's own checkpoint
(save/g2k_mcrAttn_model_kfold_train_4_0.ckpt-79, tests/golden/ckpt_attn_range.npz
made by tools/make_fixtures.py).

models/g2k_lstm_mcr.py:102-106 creates ngh = Variable(lambda * ngh) [10, 8]
and attn = Variable(ngh @ (E * Rm)) [10, 10]; in all 20 model copies the saved
attn lies in the column space of the saved ngh (relative residual of
attn - ngh pinv(ngh) attn <= 1e-12; measured <= 1.6e-15).  That pins the left
factor of the attention product.  The right factor E * Rm is not pinned: its
placeholder defaults are random and re-drawn per evaluation (Appendix B Q1),
and the checkpoint's [8, 10] Variable is no factor of it (relations that fail
are recorded in the fixture and in DESIGN.md §3).  Host code only; the same
known answer through HIP is tests/test_models_gpu.py."""
import os

import numpy as np

from oracle import g2k_ref as ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _pairs():
    z = np.load(os.path.join(GOLDEN, "ckpt_attn_range.npz"))
    return z, [(z[f"ngh{i}"], z[f"attn{i}"]) for i in range(20)]


def kat_feed(g, A):
    """The oracle / kernel inputs whose forward must return the stored attn:
    lambda = 1 and G = the stored ngh (already lambda-scaled, :102);
    Wv = [I_8 | 0], bv = 0, X = [M; 0] with M = pinv(ngh) @ attn, so E = M;
    Wr = [1 0] per row and Rel = [1; 0], so Rm = 1."""
    M = np.linalg.lstsq(g, A, rcond=None)[0]                     # [8, 10]
    X = np.zeros((12, 10))
    X[:8] = M
    Wv = np.zeros((8, 12))
    Wv[:, :8] = np.eye(8)
    Wr = np.zeros((8, 2))
    Wr[:, 0] = 1.0
    Rel = np.zeros((2, 10))
    Rel[0] = 1.0
    return dict(X=X, Rel=Rel, G=g, Wv=Wv, bv=np.zeros(10), Wr=Wr)


def test_attn_in_range_of_ngh_all_copies():
    z, pairs = _pairs()
    assert len(pairs) == 20
    for i, (g, A) in enumerate(pairs):
        assert g.shape == (10, 8) and A.shape == (10, 10)
        M = np.linalg.lstsq(g, A, rcond=None)[0]
        r = np.abs(A - g @ M).max() / np.abs(A).max()
        assert r <= 1e-12, (i, r)
        assert np.linalg.matrix_rank(g) == 8                      # the factor is informative
    # the relations that do not hold (recorded for DESIGN.md §3)
    assert z["cost_vs_E_ngh"].min() > 0.5 and z["attn_vs_ngh_E"].min() > 0.5


def test_oracle_forward_returns_the_stored_attn():
    """oracle.mcr_forward (the restatement of models/g2k_lstm_mcr.py:99-124)
    reproduces every stored attn from the stored ngh."""
    _, pairs = _pairs()
    rng = np.random.default_rng(0)
    for g, A in pairs:
        f = kat_feed(g, A)
        o = ref.mcr_forward(f["X"], f["Rel"], f["G"], f["Wv"], f["bv"], f["Wr"],
                            rng.standard_normal((24, 8)), rng.standard_normal((8, 3)), 1.0)
        assert np.abs(o["attn"] - A).max() <= 1e-12 * max(1.0, np.abs(A).max())
        np.testing.assert_array_equal(o["ngh"], g)
