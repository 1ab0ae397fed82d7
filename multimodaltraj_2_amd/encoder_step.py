"""--use_grid_lstm: the vis/loc
encoder's GridLSTMCell inside the frame loop.

The reference builds neighborhood_vis_loc_encoder (helper.py:10-75) and runs
it every frame (train.py:201-207) with ``inputs`` = the frame's input
embedding Wii @ (batch_v @ Wi) [D, D] and ``state_f00_b00_c`` = the hidden
state entering the frame [D, H] (the cell reads its first K*2u = 16 columns,
SURVEY.md Appendix C).  It then overrides the cell's outputs by feeding
``output`` / ``c_hidden_state`` and hands the INPUT placeholder on as
``st_embeddings`` (:201-207, 231), so the encoder never reaches the model:
that is the default here too (``--use_grid_lstm 0``).  With the flag the
build takes the stage's intent: st_embeddings := the cell's output, so the
model input X = [GridLSTM(inputs, h[:, :16]); vislet_emb] of a frame depends
on the hidden state and the frames of a chain become sequential (pred and
attn depend on h, unlike the default path, where only h is a chain).

The chain runs frame by frame on the GPU in ONE workgroup
(g2k_encoder_chain_f32, ABI 8): g2k_frame_embed_f32 once (every frame of
every batch), then a single launch that walks the frames — per frame the
GridLSTM cell (writing straight into that frame's X rows), the model forward
of one feed and one recurrence frame, separated by workgroup barriers — and
g2k_ade_fde_f32 over the collected predictions.  (Round 4 issued three
launches per frame from a Python loop: tests/test_encoder_chain_gpu.py checks
both bit-identical and times them.)  There is no CPU fallback.
Oracle: oracle.scene_step(encoder=) (gridlstm_cell chained in); the cell is
third-party TF contrib code, so its
parity is unpinned (row a6)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import frame_step as fs


class EncoderChain:
    """One hidden-state chain through the frames of S batches in order (the
    training leg carries ``hidden_state`` batch after batch, train.py:197-252)
    with the GridLSTM encoder stage in every frame.  ``cell``: a
    helper.GridLSTMCell (W, b, peep; feature_size * K = D columns)."""

    def __init__(self, params: fs.G2KParams, cell, *, lam=fs.LAMBDA):
        self.params, self.cell, self.lam = params, cell, lam
        if cell.feature_size * sum(cell.num_frequency_blocks) != fs.HIDDEN_LEN or \
                2 * cell.num_units * sum(cell.num_frequency_blocks) != fs.HIDDEN_LEN:
            raise ValueError("the encoder must map [D, D] inputs to [D, D] outputs (D = 16)")

    def run(self, pos, vislet, G, targets, n_active, n_frames, h, *, ped_mask=None, stride=0,
            stream=None) -> tuple:
        """pos [S, W, Nmax, 2], vislet [S, 2, Nmax], G [S, D, T], targets
        [S, F, Nmax, L, 2], n_active / n_frames [S] int32, h [1, D, H] (updated
        in place: the chain).  Returns (StepOutputs with pred [S, F, 2L, Nmax]
        (band), metrics [S, 8], attn, cost; h)."""
        dev = pos.device
        if dev.type != "cuda":
            raise ValueError("the encoder chain runs on the GPU only (no CPU fallback)")
        S, F = int(pos.shape[0]), int(targets.shape[1])
        D, Nmax = fs.HIDDEN_LEN, int(pos.shape[2])
        fs._check_dev("h", h, dev, torch.float32)
        if h.dim() != 3 or tuple(h.shape[:2]) != (1, D):
            raise ValueError("h must be one contiguous chain [1, D, H]")
        X, Rel = fs.frame_embed(self.params, pos, vislet, n_active, F, stride=stride,
                                stream=stream)
        Xe = torch.empty_like(X)            # rows D, D+1 (vislet_emb) = X's; 0..D-1 per frame
        pred = torch.zeros((S, F, 2 * fs.PRED_LEN, Nmax), device=dev)
        attn = torch.zeros((S, F, D, D), device=dev)
        cost = torch.zeros((S, F, fs.OBS_LEN, fs.OBS_LEN), device=dev)
        scratch = torch.empty((D, D), device=dev)
        c = self.cell
        for k, t in (("G", G), ("cell W", c.W), ("cell b", c.b)):
            fs._check_dev(k, t, dev, torch.float32)
        for k, t in (("n_active", n_active), ("n_frames", n_frames)):
            fs._check_dev(k, t, dev, torch.int32)
            if tuple(t.shape) != (S,):
                raise ValueError(f"{k}: shape {tuple(t.shape)}, expected {(S,)}")
        if tuple(G.shape) != (S, D, fs.OBS_LEN):
            raise ValueError(f"G: shape {tuple(G.shape)}, expected {(S, D, fs.OBS_LEN)}")
        u, fsz = int(c.num_units), int(c.feature_size)
        if tuple(c.W.shape) != (fsz + 2 * u, 3 * u) or tuple(c.b.shape) != (3 * u,):
            raise ValueError(f"cell W must be [{fsz + 2 * u}, {3 * u}] and b [{3 * u}]")
        if c.peep is not None:
            if tuple(c.peep.shape) != (4, u):
                raise ValueError(f"cell peep must be [4, {u}]")
            if c.peep.dtype != torch.float32 or c.peep.device != dev:
                raise TypeError(f"cell peep: {c.peep.dtype} on {c.peep.device}, expected "
                                f"torch.float32 on {dev}")
        peep = None if c.peep is None else c.peep.contiguous()
        W, b, Gc = c.W.contiguous(), c.b.contiguous(), G.contiguous()
        lib = _lib.load()
        d = _lib.G2KDims(S, F, fs.OBS_LEN, fs.PRED_LEN, D, int(h.shape[2]), Nmax, 0, 0)
        w = self.params.abi()
        rc = lib.g2k_encoder_chain_f32(
            ctypes.byref(d), ctypes.byref(w), fs._ptr(X), fs._ptr(Rel), fs._ptr(Gc),
            fs._ptr(n_active), fs._ptr(n_frames), W.data_ptr(), b.data_ptr(),
            None if peep is None else peep.data_ptr(), int(c.feature_size), int(c.num_units),
            fs._ptr(Xe), fs._ptr(scratch), fs._ptr(attn), fs._ptr(cost), fs._ptr(pred), fs._ptr(h),
            float(self.lam), fs._stream(stream))                    # train.py:201-207, :240-252
        _lib.check("g2k_encoder_chain_f32", rc)
        self._keep = (W, b, peep, Gc, scratch, X, Rel)
        metrics = fs.ade_fde(pred, targets, n_active, n_frames=n_frames, ped_mask=ped_mask,
                             stream=stream)                                   # :636-674
        return fs.StepOutputs(pred=pred, h=h, metrics=metrics, attn=attn, cost=cost), h
