"""DataLoader of the reference (load_traj.py), host side.

Same constructor, attributes and ``next_step()`` contract as the reference's
``DataLoader`` (load_traj.py:9-281) so that train.py / sample.py read the
same batches, with the build decisions of SURVEY.md Appendix B:

* Q8  — the data root is a parameter (``data_root``), not a hard-coded path;
* Q18 — ``sel=None`` selects file 0 instead of prompting with ``input()``;
* the frame dict (``trajectories``) is the one the reference READS: with
  ``infer=False`` it loads ``trajectories_0.cpkl`` whenever that file exists
  (load_traj.py:95-112), and each shipped pickle is frame_preprocess
  (load_traj.py:234-256) over the WHOLE CSV — its bytes equal
  ``pickle.dumps`` of that dict (tests/test_frame_dict.py, the file's sha256 in
  tests/golden/data_*.npz), while the walk's bound ``max(self.frameList)``
  (:163) and ``num_batches`` (:104) stay the 70 % split's.  Without a pickle
  (eth/univ; every ``infer=True`` loader) the reference builds the dict over
  the split it loaded.  The dict is rebuilt from the CSV here; the pickles are
  never unpickled (``frame_dict="whole" | "split"``, default: as the
  reference would find it);
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

class TrajIndex:
    """Native index over the frame dict's columns (g2k_traj_create;
    csrc/g2k_walk.cpp): the dict's keys and rows, and the reference's batch
    walk over them.
    Host code only: usable without a GPU."""

    def __init__(self, frames, peds, diff, walk_max=None):
        """``frames`` / ``peds``: rows 0 / 1 of the columns the frame dict
        spans; ``walk_max``: next_step's max(self.frameList) (default: the
        largest of ``frames``)."""
        from . import _lib
        self._lib = _lib.load()
        self.frames = np.ascontiguousarray(frames, dtype=np.float64)
        peds = np.ascontiguousarray(peds, dtype=np.float64)
        self.cols = int(self.frames.shape[0])
        self.walk_max = float(self.frames.max() if walk_max is None else walk_max)
        self._h = self._lib.g2k_traj_create(self.frames.ctypes.data, peds.ctypes.data, self.cols,
                                            int(diff), self.walk_max)
        if not self._h:
            _lib.check("g2k_traj_create", -1)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.g2k_traj_destroy(h)

    def next_step(self, frame_pointer, batch_size, obs_len):
        """-> (batch keys [k] float64, drawn columns, columns per draw, new
        frame pointer); load_traj.py:153-224."""
        import ctypes
        from . import _lib
        cap = max(4 * batch_size, 64)
        keys = np.empty(cap, np.float64)
        nk, nd, nxt = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_double()
        dlen = np.empty(cap * batch_size, np.int64)
        rc = self._lib.g2k_traj_next_step(self._h, float(frame_pointer), batch_size, obs_len,
                                          keys.ctypes.data, cap, ctypes.byref(nk), None, 0,
                                          dlen.ctypes.data, ctypes.byref(nd), ctypes.byref(nxt))
        _lib.check("g2k_traj_next_step", rc)
        dlen = dlen[:nd.value]
        cols = np.empty(max(int(dlen.sum()), 1), np.int64)
        rc = self._lib.g2k_traj_next_step(self._h, float(frame_pointer), batch_size, obs_len,
                                          keys.ctypes.data, cap, ctypes.byref(nk), cols.ctypes.data,
                                          cols.size, dlen.ctypes.data, ctypes.byref(nd),
                                          ctypes.byref(nxt))
        _lib.check("g2k_traj_next_step", rc)
        return keys[:nk.value].copy(), cols, dlen, nxt.value

    def sample_scenes(self, frame_pointers, nmax, batch_size=16, obs_len=8, pred_len=12):
        """sample.py:138-164 scenes for many frame pointers at once ->
        dict(pos_col [n, 8, nmax], tgt_col [n, nmax, 12], n_nodes [n],
        n_keys [n], next_pointer [n]) (g2k_traj_sample_scenes)."""
        from . import _lib
        fps = np.ascontiguousarray(frame_pointers, dtype=np.float64).reshape(-1)
        n = int(fps.size)
        out = dict(pos_col=np.empty((n, 8, nmax), np.int32), tgt_col=np.empty((n, nmax, 12), np.int32),
                   n_nodes=np.empty(n, np.int32), n_keys=np.empty(n, np.int32),
                   next_pointer=np.empty(n, np.float64))
        rc = self._lib.g2k_traj_sample_scenes(
            self._h, fps.ctypes.data, n, batch_size, obs_len, pred_len, nmax,
            out["pos_col"].ctypes.data, out["tgt_col"].ctypes.data, out["n_nodes"].ctypes.data,
            out["n_keys"].ctypes.data, out["next_pointer"].ctypes.data)
        _lib.check("g2k_traj_sample_scenes", rc)
        return out


DATA_DIRS = ["eth/hotel/", "eth/univ/", "ucy/zara/zara01/", "ucy/zara/zara02/", "ucy/univ/",
             "town_center.csv", "annotation_tc.txt"]     # load_traj.py:25-33


class DataLoader:
    def __init__(self, args, datasets=(0, 1, 2, 3, 4, 5, 6), sel=None, start=0,
                 processFrame=False, infer=False, data_root=None, raw_data=None,
                 frame_dict=None):
        """load_traj.py:11-104.  ``raw_data`` (the CSV array) may be passed
        directly (tests, fixtures) instead of reading ``data_root``.
        ``frame_dict``: "whole" (the dict over the whole CSV: what the shipped
        trajectories_0.cpkl holds) or "split" (frame_preprocess over the loaded
        split: what the reference builds when no pickle exists); default: "whole"
        when the reference would load a pickle — from ``data_root``, when
        ``<dir>/trajectories_<sel>.cpkl`` exists (``val_...`` with infer,
        load_traj.py:72-95); with ``raw_data``, unless ``infer``."""
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
        if frame_dict is None:
            if raw_data is not None:
                frame_dict = "split" if infer else "whole"
            else:
                name = ("val_trajectories_{0}.cpkl" if infer else "trajectories_{0}.cpkl")
                pk = os.path.join(self.current_dir, name.format(int(self.dataset_pointer)))
                frame_dict = "whole" if os.path.exists(pk) else "split"   # :95-103
        if frame_dict not in ("whole", "split"):
            raise ValueError(f"frame_dict must be 'whole' or 'split', not {frame_dict!r}")
        self.frame_dict = frame_dict
        if raw_data is not None:
            self._set_raw(np.asarray(raw_data, dtype=np.float64), val=infer)
        elif os.path.isdir(self.current_dir):
            files = sorted(glob.glob(os.path.join(self.current_dir, "*.csv")))
            if not files:
                raise FileNotFoundError(f"no CSV under {self.current_dir}")
            self.load_dataset(files[int(self.dataset_pointer)], val=infer)
        else:
            # a file entry of the list (town_center.csv, annotation_tc.txt):
            # loaded as is (load_traj.py:89-92); the reference's data/ does not
            # ship them, so this raises FileNotFoundError as np.genfromtxt does
            if not os.path.exists(self.current_dir):
                raise FileNotFoundError(f"{self.current_dir} not found (load_traj.py:89-92)")
            self.load_dataset(self.current_dir, val=infer)
        self._traj = None          # the frame dict, built on first use
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
        self._fmax = self.frameList.max()          # max(self.frameList), load_traj.py:163
        # the columns the frame dict spans (see the module docstring)
        self.dict_data = raw if self.frame_dict == "whole" else src
        self.index = TrajIndex(self.dict_data[0], self.dict_data[1], self.diff, walk_max=self._fmax)

    @property
    def trajectories(self):
        """The frame dict {frame: [{ped: [x, y]}, ...]} (load_traj.py:234-256),
        built on first use (the native index plans the walk without it)."""
        if self._traj is None:
            self._traj = self.frame_preprocess()
        return self._traj

    def frame_preprocess(self, data_file=None, seed=0):
        """load_traj.py:234-256 over the dict's columns (``dict_data``):
        {frame: [{ped: [x, y]}, ...]}; every frame value is a key (empty dict),
        frames seed + k*diff <= max get their peds."""
        d = self.dict_data
        frame_data = {i: {} for i in d[0]}
        # the rows of each frame index in file order, grouped in one pass (the
        # reference rescans every row per frame: same lists, O(rows) here)
        rows = {}
        for (ind, ped, px, py) in np.transpose(d[0:4]):
            rows.setdefault(ind, []).append({ped: [px, py]})
        fp = self.seed
        fmax = d[0].max()
        while fp <= fmax:
            frame_data[fp] = rows.get(fp, [])
            fp += self.diff
        return frame_data

    def frame_dict_pickle(self):
        """The bytes frame_preprocess writes for this dict (load_traj.py:254-256:
        ``pickle.dump(frame_data, f, protocol=2)``) as the numpy 1.x the
        reference ran under writes them: a scalar's reduce names
        ``numpy.core.multiarray`` and the float64 dtype's constructor arguments
        are the ints 0 / 1 (numpy >= 2 writes ``numpy._core`` and bools).  For
        the shipped datasets these are the bytes of ``trajectories_0.cpkl``."""
        import pickle
        b = pickle.dumps(self.trajectories, protocol=2)
        b = b.replace(b"cnumpy._core.multiarray\nscalar\n", b"cnumpy.core.multiarray\nscalar\n")
        return b.replace(b"X\x02\x00\x00\x00f8q\x03\x89\x88\x87",
                         b"X\x02\x00\x00\x00f8q\x03K\x00K\x01\x87", 1)

    def next_step(self, targets=None):
        """Batch of frame dicts + target lists; contract of load_traj.py:153-224.

        The walk itself (which keys the batch holds, which frames are drawn
        as targets, the new frame pointer) is planned natively
        (``TrajIndex.next_step``, csrc/g2k_walk.cpp); this builds the
        reference's dicts from the plan: the batch's frames in x_batch order,
        and for every draw each of the drawn frame's pedestrians' positions
        appended pred_len times (quirk Q11; the position objects are the frame
        dict's own, as the reference appends them)."""
        tgt = {} if targets is None else targets
        keys, draw_cols, draw_len, fp = self.index.next_step(self.frame_pointer, self.batch_size,
                                                             self.obs_len)
        batch = {int(k): self.trajectories[k] for k in keys}
        reps = int(self.pred_len)
        at = 0
        for n in draw_len:
            if n == 0:
                continue
            entries = self.trajectories[self.dict_data[0, draw_cols[at]]]
            at += n
            ids = [int(next(iter(e))) for e in entries]
            if len(set(ids)) == len(ids):
                for pid, e in zip(ids, entries):
                    xy = next(iter(e.values()))
                    if pid in tgt:
                        tgt[pid].extend([xy] * reps)
                    else:
                        tgt[pid] = [xy] * reps
            else:                       # a pedestrian twice in one frame: the exact order
                for _ in range(reps):
                    for pid, e in zip(ids, entries):
                        tgt.setdefault(pid, []).append(next(iter(e.values())))
        self.frame_pointer = fp
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
