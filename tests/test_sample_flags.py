"""sample.py's flags (sample.py:89-106) on top of argParser.py's: same names
and defaults as the reference, and dataset 5 (town_center.csv, absent from
the reference's data/) failing as the reference's loader does (CPU only)."""
import pytest

from multimodaltraj_2_amd import sample
from multimodaltraj_2_amd.load_traj import DataLoader


def test_sample_flag_defaults_match_reference():
    a = sample.parse_args([])
    assert (a.obs_length, a.pred_length, a.test_dataset, a.epoch) == (8, 12, 5, 2)
    # argParser.py defaults the sample path reads
    assert (a.num_freq_blocks, a.rnn_size, a.grid_size, a.lambda_param) == (10, 128, 4, 0.0005)
    assert sample.parse_args(["--test_dataset", "2"]).test_dataset == 2


def test_default_dataset_is_town_center_and_absent(tmp_path):
    a = sample.parse_args(["--data_root", str(tmp_path)])
    with pytest.raises(FileNotFoundError, match="town_center.csv"):
        DataLoader(a, datasets=[0, 1, 2, 3, 4, 5], start=a.test_dataset, sel=0,
                   data_root=a.data_root)
