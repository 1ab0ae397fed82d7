"""The frame dict the reference reads (load_traj.py:95-112): for every dataset
that ships trajectories_0.cpkl it is frame_preprocess (load_traj.py:234-256)
over the WHOLE CSV, not over the 70 % training split the walk is bounded by.

Pinned without unpickling anything: the package's dict, re-pickled the way the
reference wrote it (protocol 2, numpy 1.x scalar/dtype encoding), must hash to
the sha256 of the shipped pickle's bytes (recorded in tests/golden/data_*.npz
by tools/make_fixtures.py, which also compared the bytes in full).  Host code
only."""
import glob
import hashlib
import os
from types import SimpleNamespace

import numpy as np
import pytest

from multimodaltraj_2_amd.load_traj import DataLoader

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ARGS = SimpleNamespace(batch_size=16, seq_length=12, pred_len=12, obs_len=8)
FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "data_*.npz")))
# key counts of the shipped pickles (whole-CSV dicts)
WHOLE_KEYS = {"eth_hotel": 3134, "zara01": 1127, "zara02": 1315, "ucy_univ": 676}


def _name(path):
    return os.path.basename(path)[5:-4]


@pytest.mark.parametrize("path", FIXTURES, ids=[_name(p) for p in FIXTURES])
def test_rebuilt_dict_is_the_pickled_dict(path):
    z = np.load(path)
    name, mode = _name(path), str(z["frame_dict"])
    if mode == "whole":
        dl = DataLoader(ARGS, raw_data=z["raw_data"])      # default with raw data: the pickled dict
        assert dl.frame_dict == "whole"
        assert len(dl.trajectories) == int(z["dict_keys"]) == WHOLE_KEYS[name]
        assert hashlib.sha256(dl.frame_dict_pickle()).hexdigest() == str(z["pickle_sha256"])
    else:                                                   # eth/univ: no pickle ships
        assert name not in WHOLE_KEYS
        dls = DataLoader(ARGS, raw_data=z["raw_data"], frame_dict="split")
        assert len(dls.trajectories) == int(z["dict_keys"])


@pytest.mark.parametrize("path", FIXTURES, ids=[_name(p) for p in FIXTURES])
def test_walk_bound_is_the_split(path):
    """The dict spans the whole CSV, the walk's max(self.frameList) (:163) and
    num_batches (:104) stay the training split's."""
    z = np.load(path)
    raw = z["raw_data"]
    dl = DataLoader(ARGS, raw_data=raw, frame_dict=str(z["frame_dict"]))
    split = raw[:, :int(raw.shape[1] * 0.7)]
    assert dl.index.walk_max == split[0].max()
    assert dl.num_batches == int(z["num_batches"]) == int(split.shape[1] / 12 / 16)
    assert dl.index.cols == (raw.shape[1] if str(z["frame_dict"]) == "whole" else split.shape[1])
    # keys past the split exist in the whole dict (zara02's boundary frame keeps all its peds)
    if str(z["frame_dict"]) == "whole":
        on_grid = split[0][(split[0] - split[0, 0]) % ARGS.obs_len == 0]
        last = on_grid[-1]                                  # the split's last grid frame
        full = [r for r in np.transpose(raw[0:4]) if r[0] == last]
        assert len(dl.trajectories[last]) == len(full)


def test_auto_mode_follows_the_pickle(tmp_path):
    """From a data root, "whole" exactly when trajectories_<sel>.cpkl exists
    (load_traj.py:95), "split" otherwise and for infer loaders (val_...)."""
    z = np.load(os.path.join(GOLDEN, "data_zara01.npz"))
    d = tmp_path / "ucy" / "zara" / "zara01"
    d.mkdir(parents=True)
    np.savetxt(d / "vis_body.csv", z["raw_data"], delimiter=",")
    dl = DataLoader(ARGS, datasets=[0, 1, 2, 3, 4, 5], start=2, sel=0, data_root=str(tmp_path))
    assert dl.frame_dict == "split"
    (d / "trajectories_0.cpkl").write_bytes(b"")
    dl = DataLoader(ARGS, datasets=[0, 1, 2, 3, 4, 5], start=2, sel=0, data_root=str(tmp_path))
    assert dl.frame_dict == "whole"
    dl = DataLoader(ARGS, datasets=[0, 1, 2, 3, 4, 5], start=2, sel=0, data_root=str(tmp_path),
                    infer=True)
    assert dl.frame_dict == "split"
