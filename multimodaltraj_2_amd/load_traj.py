"""DataLoader of the reference (load_traj.py), host side.

Same constructor, attributes and ``next_step()`` contract as the reference's
``DataLoader`` (load_traj.py:9-281) so that train.py / sample.py read the
same batches, with the build decisions of SURVEY.md Appendix B:

* Q8  — the data root is a parameter (``data_root``), not a hard-coded path;
* Q18 — ``sel=None`` selects file 0 instead of prompting with ``input()``;
* the frame dict (``trajectories``) is always rebuilt from the CSV with the
  reference's own frame_preprocess arithmetic (load_traj.py:234-256); the
  pickled ``trajectories_0.cpkl`` files are never loaded;
* ``next_step``'s mutable default ``targets={}`` (load_traj.py:153) is
  never mutated by the reference (its first insertion rebinds ``targets`` to
  a new dict, :216-217), so every call starts from an empty dict: ``None``
  default here, same rebinding rule.

Parity: tests/test_data_path.py against fixtures produced by running the
reference's own load_traj/networkx_graph (tools/make_fixtures.py).
"""
from __future__ import annotations

import glob
import math
import os

import numpy as np

DATA_DIRS = ["eth/hotel/", "eth/univ/", "ucy/zara/zara01/", "ucy/zara/zara02/", "ucy/univ/",
             "town_center.csv", "annotation_tc.txt"]     # load_traj.py:25-33


class DataLoader:
    def __init__(self, args, datasets=(0, 1, 2, 3, 4, 5, 6), sel=None, start=0,
                 processFrame=False, infer=False, data_root=None, raw_data=None):
        """load_traj.py:11-104.  ``raw_data`` (the CSV array) may be passed
        directly (tests, fixtures) instead of reading ``data_root``."""
        self.data_dirs = [os.path.join(data_root or "", d) for d in DATA_DIRS]
        self.used_data_dirs = [self.data_dirs[x] for x in datasets]
        self.infer = infer
        self.numDatasets = len(self.data_dirs)
        self.data_dir = data_root
        self.batch_size = args.batch_size
        self.seq_length = args.seq_length
        self.pred_len = args.pred_len
        self.obs_len = args.obs_len
        self.diff = self.obs_len
        self.current_dir = self.used_data_dirs[start]
        self.dataset_pointer = 0 if sel is None else sel
        if raw_data is not None:
            self._set_raw(np.asarray(raw_data, dtype=np.float64), val=infer)
        else:
            files = sorted(glob.glob(os.path.join(self.current_dir, "*.csv")))
            if not files:
                raise FileNotFoundError(f"no CSV under {self.current_dir}")
            self.load_dataset(files[int(self.dataset_pointer)], val=infer)
        self.trajectories = self.frame_preprocess()
        self.num_batches = int((len(self.frameList) / self.seq_length) / self.batch_size)

    # load_traj.py:114-150
    def load_dataset(self, data_file, val=False):
        self._set_raw(np.genfromtxt(fname=data_file, delimiter=","), val=val)

    def _set_raw(self, raw, val=False):
        self.raw_data = raw
        self.len = raw.shape[1]
        self.max = int(raw.shape[1] * 0.7)
        self.val_max = int(raw.shape[1] * 0.3)
        self.val_data = raw[:, self.max:self.max + self.val_max]
        self.tr_data = raw[:, 0:self.max]
        src = self.val_data if val else self.tr_data
        self.frameList = src[0, :]
        self.pedsPerFrameList = src[0:4, :]
        # ETH CSVs have 4 rows: no vislet rows (Appendix B Q14 -> zeros)
        self.vislet = src[4:6, :] if src.shape[0] >= 6 else np.zeros((2, src.shape[1]))
        self.seed = self.frameList[0]
        self.frame_pointer = self.seed

    def frame_preprocess(self, data_file=None, seed=0):
        """load_traj.py:234-256: {frame: [{ped: [x, y]}, ...]}; every frame of
        frameList is a key (empty dict), frames seed + k*diff get their peds."""
        frame_data = {i: {} for i in self.frameList}
        # the rows of each frame index in file order, grouped in one pass (the
        # reference rescans every row per frame: same lists, O(rows) here)
        rows = {}
        for (ind, ped, px, py) in np.transpose(self.pedsPerFrameList):
            rows.setdefault(ind, []).append({ped: [px, py]})
        fp = self.frame_pointer
        fmax = self._fmax = max(self.frameList)
        while fp <= fmax:
            frame_data[fp] = rows.get(fp, [])
            fp += self.diff
        return frame_data

    def next_step(self, targets=None):
        """Batch of frame dicts + target lists; contract of load_traj.py:153-224.

        Up to batch_size + 1 passes; each pass appends the frames
        frame_pointer, +diff, ... (batch_size keys, stopping at the first
        missing key) to a growing window, then walks the window in insertion
        order with a single cursor that the reference advances once per
        visited key and once more per target draw (its ``iter_traj``).  Every
        obs_len-th visit draws the frame under the cursor and appends each of
        its pedestrians' positions pred_len times to ``targets`` (quirk Q11).
        A pass stops the walk when the cursor runs out; the last key touched
        feeds the end-of-data test of the next pass."""
        tgt = {} if targets is None else targets
        batch, window = {}, {}
        visits = 1                                   # `pc`, kept across passes
        fmax = self._fmax
        last = self.frame_pointer
        span = self.batch_size * self.obs_len
        for _ in range(self.batch_size + 1):
            if fmax - (last + 1) <= 0:
                break
            # the log-scale test of :175-177 always holds once the gap is > 0
            for key in range(int(self.frame_pointer), int(self.frame_pointer + span), self.diff):
                last = key
                if key not in self.trajectories:
                    break
                window[key] = self.trajectories[key]
            order = list(window)
            cursor = 0
            for key in order:
                last = key
                frame = self.trajectories[key]
                if len(frame):
                    batch[key] = frame
                    if visits % self.obs_len == 0:
                        if cursor >= len(order):
                            break
                        drawn = self.trajectories[order[cursor]]
                        cursor += 1
                        for _rep in range(int(self.pred_len)):
                            for entry in drawn:
                                (pid, xy), = entry.items()
                                pid = int(pid)
                                if not tgt:
                                    tgt = {pid: [xy]}      # rebinding, as the reference
                                elif pid in tgt:
                                    tgt[pid].append(xy)
                                else:
                                    tgt[pid] = [xy]
                visits += 1
                if cursor >= len(order):
                    break
                cursor += 1
            self.frame_pointer += self.diff
        return batch, tgt, self.frame_pointer

    def tick_frame_pointer(self, valid=False, incr=8):
        if not valid:
            self.frame_pointer += incr

    def reset_data_pointer(self, valid=False, dataset_pointer=0, frame_pointer=0):
        if not valid:
            self.frame_pointer = self.seed
        else:
            self.dataset_pointer = dataset_pointer
            self.frame_pointer = frame_pointer
