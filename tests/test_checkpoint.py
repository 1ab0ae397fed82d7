"""TF tensor-bundle reader/writer (multimodaltraj_2_amd/checkpoint.py;
SURVEY.md §8(f) row 3, Appendix D).  Pinned byte for byte by the reference's
own checkpoint save/g2k_mcr_model_val_0.ckpt-0 (copied as data into
tests/golden/ckpt_val0.*): decoding then re-encoding it reproduces both files
exactly (table layout, restart points, masked CRC32Cs, key successor, footer).
When /root/reference is present (build container only) all eight reference
checkpoints are re-encoded the same way."""
import glob
import os

import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import checkpoint as ck
from multimodaltraj_2_amd import frame_step as fs

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ckpt_val0")


def _same_bytes(src, dst):
    for ext in (".index", ".data-00000-of-00001"):
        assert open(src + ext, "rb").read() == open(dst + ext, "rb").read(), ext


def test_crc32c_known_answer():
    assert ck.crc32c(b"123456789") == 0xE3069283


def test_reencode_reference_checkpoint_byte_exact(tmp_path):
    t, meta = ck.read_bundle(GOLD, with_meta=True)
    assert len(t) == 17
    assert t["grid_lstm_cell/W_f_0_0"].shape == (8, 6)
    data = open(GOLD + ".data-00000-of-00001", "rb").read()
    for k, (o, n, c) in meta.items():
        assert c == ck.mask_crc(ck.crc32c(data[o:o + n])), k
    out = str(tmp_path / "re")
    ck.write_bundle(out, t)
    _same_bytes(GOLD, out)


@pytest.mark.skipif(not os.path.isdir("/root/reference/save"), reason="reference checkpoints absent")
def test_reencode_all_reference_checkpoints(tmp_path):
    prefixes = sorted(p[:-6] for p in glob.glob("/root/reference/save/*.index"))
    assert len(prefixes) == 8
    for i, prefix in enumerate(prefixes):
        out = str(tmp_path / f"c{i}")
        ck.write_bundle(out, ck.read_bundle(prefix))
        _same_bytes(prefix, out)


def test_params_roundtrip(tmp_path):
    p = fs.init_params(12, seed=3)
    prefix = str(tmp_path / "save" / "g2k_model.ckpt-50")
    names = ck.save_params(prefix, p)
    assert names == sorted(names)
    q = ck.load_params(prefix)
    for k in ("Wi", "Wii", "Wv", "bv", "Wr", "Wc", "Wo"):
        assert torch.equal(getattr(p, k), getattr(q, k))
    t = ck.read_bundle(prefix)
    assert t["krnl_weights/Wo"].dtype == np.float32 and t["krnl_weights/Wo"].shape == (8, 12)
