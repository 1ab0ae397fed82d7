"""CPU: bench.py's roofline arithmetic.  The per-frame
flops reproduce the survey's F_frame table at Nmax, the bound follows the
launch's intensity against the FP32 ridge (19.7 flop/B), and both fractions
are carried."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, FRAMES_PER_SCENE, make_batch  # noqa: E402


@pytest.mark.parametrize("n,H,want", [(32, 128, 130_848), (64, 128, 155_680),
                                      (64, 256, 241_696), (256, 256, 390_688)])
def test_survey_f_frame_table(n, H, want):
    assert bench.flops_per_frame(n, H) == want
    assert bench.flops_per_frame(n, H, grid_lstm=True) == want + 8_064


def test_survey_terms_sum():
    """The per-term breakdown of §8(d) (D 16, T 8) gives 776 N + 19,968 +
    672 H; the survey rounds the constant to 20,000."""
    D, T = 16, 8
    for n, H in ((1, 128), (17, 256)):
        terms = (2 * T * n * D + 2 * D * D * T + 4 * n * D + 2 * T * (D + 2) * D + T * D
                 + 4 * T * D + 2 * D * D * T + T * D + 2 * D * T * T + 48 * T * T + 48 * T * n
                 + 5 * D * D + 2 * D * D * H + 10 * D * H + 72 * n)
        assert terms + 32 == bench.flops_per_frame(n, H)


def test_ridge_and_bound():
    assert bench.RIDGE == pytest.approx(19.66, abs=0.01)
    hb = bench.roofline(1e6, 10e6, 1e-6, 0.5e-6)          # 10 flop/B: HBM
    assert hb["bound"] == "hbm" and hb["unit"] == "GB/s"
    assert hb["achieved"] == pytest.approx(1e6 / 1e-6 / 1e9)
    assert hb["frac"] == pytest.approx(hb["frac_hbm"])
    assert hb["frac_hbm_per_step"] == pytest.approx(2 * hb["frac_hbm"])
    cb = bench.roofline(1e6, 30e6, 1e-6, 1e-6)            # 30 flop/B: compute
    assert cb["bound"] == "mfma" and cb["unit"] == "TFLOP/s" and cb["peak"] == 157.3
    assert cb["frac"] == pytest.approx(30e6 / 1e-6 / 1e12 / 157.3)
    assert cb["frac"] == pytest.approx(cb["frac_flops"])


def test_headline_launch_is_compute_bound():
    """eth_hotel_synth (BASELINE configs[1]): ~28 flop/B at its batch's mean
    active N (U{2..32}) — above the ridge (VERDICT r5 What's weak 2)."""
    cfg = CONFIGS["eth_hotel_synth"]
    b = make_batch(cfg["S"], cfg["Nmax"], cfg["H"], F=FRAMES_PER_SCENE, seed=1)
    pbytes = 4 * (cfg["Nmax"] * 16 + 16 * 8 + 8 * 18 + 16 + 8 * 2 + 24 * 8 + 8 * cfg["Nmax"])
    ab = bench.algorithmic_bytes(b, cfg["H"], pbytes)
    af = bench.algorithmic_flops(b, cfg["H"])
    assert af == int((FRAMES_PER_SCENE * (776 * b.n_active.astype(np.int64) + 20_000
                                          + 672 * cfg["H"])).sum())
    assert 26 < af / ab < 31
    r = bench.roofline(ab, af, 19.14e-6, 14.4e-6)
    assert r["bound"] == "mfma" and 0.15 < r["frac"] < 0.25


def test_train_flops_add_the_gradient():
    b = make_batch(8, 32, 128, F=FRAMES_PER_SCENE, seed=2)
    P = 1000
    fwd = bench.algorithmic_flops(b, 128)
    n = b.n_active.astype(np.int64)
    bwd = int((FRAMES_PER_SCENE * (72 * n + 768 * n + 320 * n + 25_728)).sum())
    assert bench.train_algorithmic_flops(b, 128, P) == fwd + bwd + 8 * (P + 2) + 8 * P
    assert bench.train_algorithmic_flops(b, 128, P, "nll") > bench.train_algorithmic_flops(b, 128, P)
