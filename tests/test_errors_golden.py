"""a9 pinned by the reference's OWN error code: tests/golden/errors_*.npz hold
the outputs of get_mean_error (sample.py:21-82), the validation frame block
(train.py:636-662), its per-batch reductions (train.py:668-674) and the
training-log block (train.py:254-276), executed by tools/make_error_fixtures.py
on real walk batches (the statements are loaded from the reference source
with ``ast`` at generation time and run with real NumPy).  Here the float64
oracle restatement must reproduce them to 1e-12 (CPU only)."""
import glob
import os

import numpy as np
import pytest

from oracle import g2k_ref as ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
FILES = sorted(glob.glob(os.path.join(GOLDEN, "errors_*.npz")))
TOL = 1e-12


def rebuild_dict(z, q):
    """The stored part of a target dict (first keys in insertion order, true
    lengths, first 12 points; entries past the stored points are NaN so a read
    beyond what the reference reads would show) padded with never-read keys
    to the dict's true size K (the short-target divisor len(target_traj))."""
    keys, lens, heads, K = z[q + "keys"], z[q + "lens"], z[q + "heads"], int(z[q + "K"])
    td = {}
    for k, ln, hd in zip(keys, lens, heads):
        a = np.full((int(ln), 2), np.nan)
        m = min(int(ln), 12)
        a[:m] = hd[:m]
        td[int(k)] = a
    j = -1
    while len(td) < K:
        td[j] = np.full((12, 2), np.nan)
        j -= 1
    return td


def cases(z):
    return range(int(z["val_count"]))


def rel_close(got, want, tol=TOL):
    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    assert got.shape == want.shape, (got.shape, want.shape)
    if got.size == 0:
        return
    err = np.abs(got - want) / np.maximum(1.0, np.abs(want))
    assert float(err.max()) <= tol, float(err.max())


def test_fixtures_present_and_cover_the_branches():
    assert len(FILES) == 4
    n_short = n_keyerr = n_l5_diff = 0
    for f in FILES:
        z = np.load(f)
        assert int(z["val_count"]) >= 8 and int(z["gm_count"]) >= 4
        for c in cases(z):
            p = f"val{c}_"
            n_short += int(np.sum(z[p + "short_lens"][:int(z[p + "n"])] < 12))
            n = int(z[p + "n"])
            present = sum(1 for i in range(1, n) if i in set(z[p + "keys"].tolist()))
            n_keyerr += (n - 1) - present
            if np.isfinite(z[p + "fde_b"]) and z[p + "nb"] != n:
                n_l5_diff += 1
    assert n_short > 20          # the short-target branch (train.py:642-646)
    assert n_keyerr > 20         # training-log rows skipped by KeyError (train.py:274-276)
    assert n_l5_diff > 4         # the two FDE divisors differ (train.py:671-674)


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p))
@pytest.mark.parametrize("tag", ["", "short_"])
def test_validation_errors_match_reference_code(path, tag):
    z = np.load(path)
    for c in cases(z):
        p = f"val{c}_"
        n, nb = int(z[p + "n"]), int(z[p + "nb"])
        td = rebuild_dict(z, p + tag)
        cv_err, fde = [], []
        for _ in range(nb):                                   # for frame in batch
            e, f = ref.validation_frame_errors(z[p + "pred"], td, n)
            cv_err += e
            fde += f
        rel_close(cv_err, z[p + tag + "cv_err"])
        rel_close(np.reshape(fde, (-1, 2)), z[p + tag + "fde"])
        for l, key in ((2, "b"), (5, "b5")):
            a, fb = ref.validation_batch_errors(cv_err, fde, l, n, nb)
            want_a, want_f = float(z[p + tag + "ade_" + key]), float(z[p + tag + "fde_" + key])
            assert (a is None) == np.isnan(want_a) and (fb is None) == np.isnan(want_f)
            if a is not None:
                rel_close(a, want_a)
                rel_close(fb, want_f)


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p))
def test_validation_sums_match_reference_code(path):
    """The metric-sum form the kernels write ({sum ade, count, sum |fde|^2, ...,
    frames}) reduced by batch_metrics gives the reference's per-batch values
    (full-length targets: the only lists the loader produces, quirk Q11)."""
    z = np.load(path)
    for c in cases(z):
        p = f"val{c}_"
        n, nb = int(z[p + "n"]), int(z[p + "nb"])
        td = rebuild_dict(z, p)
        m = np.zeros(8)
        P_ = np.transpose(z[p + "pred"], (2, 1, 0))
        for _ in range(nb):
            for i, itr in zip(range(n), iter(td)):
                e, f = ref.validation_errors(P_[i], td[itr])
                m[0] += e
                m[1] += 1
                m[2] += float(f @ f)
            m[5] += 1
        for l, key in ((2, "b"), (5, "b5")):
            a, fb = ref.batch_metrics(m, leave_dataset=l, num_nodes=n)
            rel_close(a, z[p + "ade_" + key])
            rel_close(fb, z[p + "fde_" + key])


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p))
def test_train_log_vectors_match_reference_code(path):
    z = np.load(path)
    for c in cases(z):
        p = f"val{c}_"
        n, nb = int(z[p + "n"]), int(z[p + "nb"])
        td = rebuild_dict(z, p)
        euc, fde = [], []
        for _ in range(nb):
            e, f = ref.train_log_errors(z[p + "pred"], td)
            euc += e
            fde += f
        rel_close(np.reshape(euc, (-1, 12, 2)), z[p + "tl_euc"])
        rel_close(np.reshape(fde, (-1, 2)), z[p + "tl_fde"])
        assert int(z[p + "tl_num_end_targets"]) == nb * max(0, min(n - 1, int(z[p + "K"])))
        assert int(z[p + "tl_num_targets"]) == nb * n


@pytest.mark.parametrize("path", FILES, ids=lambda p: os.path.basename(p))
def test_get_mean_error_matches_reference_code(path):
    z = np.load(path)
    for g in range(int(z["gm_count"])):
        ct = np.transpose(z[f"gm{g}_pred"], (2, 1, 0))
        for v in range(int(z[f"gm{g}_variants"])):
            q = f"gm{g}_{v}_"
            ade, fde, cnt = ref.get_mean_error(ct, z[f"gm{g}_true"], int(z[q + "obs"]),
                                               int(z[q + "maxped"]))
            rel_close(ade, z[q + "ade"])
            rel_close(fde, z[q + "fde"])
            assert cnt == int(z[q + "counter"])
