import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


def close(got, ref, tol=1e-4):
    """SURVEY.md finding 7 / §8(d): |got - ref| <= tol * max(1, |ref|)."""
    import numpy as np
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    err = np.abs(got - ref) / np.maximum(1.0, np.abs(ref))
    return float(err.max()) if err.size else 0.0


def close_h(got, ref, rtol=1e-5, atol=1e-8):
    """The hidden state (rows of As @ softmax(h) sum to one, so entries are
    ~1/H): |got - ref| <= rtol * |ref| + atol, every entry."""
    import numpy as np
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, (got.shape, ref.shape)
    return bool(np.all(np.abs(got - ref) <= rtol * np.abs(ref) + atol))


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from multimodaltraj_2_amd import _lib
    if os.environ.get("G2K_TEST_LIB"):   # development A/B: a side build (tools/build_lib_variant.sh)
        _lib._lib = _lib.load(os.environ["G2K_TEST_LIB"])
    _lib.load()   # fails loudly if the HIP library is missing
    return torch.device("cuda:0")


FIXTURE_DIRS = {"eth_hotel": "eth/hotel/", "zara01": "ucy/zara/zara01/",
                "zara02": "ucy/zara/zara02/", "ucy_univ": "ucy/univ/"}


def write_data_root(root, names=tuple(FIXTURE_DIRS)):
    """A data root laid out as the reference's data/ (load_traj.py:25-33)
    holding the committed raw CSV arrays (tests/golden/data_*.npz), written
    with 17 significant digits so np.genfromtxt reads back the same float64."""
    import numpy as np
    for n in names:
        d = os.path.join(str(root), FIXTURE_DIRS[n])
        os.makedirs(d, exist_ok=True)
        raw = np.load(os.path.join(ROOT, "tests", "golden", f"data_{n}.npz"))["raw_data"]
        np.savetxt(os.path.join(d, "data.csv"), raw, delimiter=",", fmt="%.17g")
    return str(root)


@pytest.fixture(scope="session")
def data_root(tmp_path_factory):
    return write_data_root(tmp_path_factory.mktemp("data"))
