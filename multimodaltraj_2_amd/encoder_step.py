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

The chain runs frame by frame on the GPU: g2k_frame_embed_f32 once (every
frame of every batch), then per frame g2k_gridlstm_f32 (the cell, writing
straight into that frame's X rows) -> g2k_mcr_forward_f32 (one feed) ->
g2k_frame_recurrence_f32 (one frame), and g2k_ade_fde_f32 over the collected
predictions.  There is no CPU fallback.  Oracle: oracle.scene_step(encoder=)
(gridlstm_cell chained in); the cell is third-party TF contrib code, so its
parity is unpinned (row a6)."""
from __future__ import annotations

import numpy as np
import torch

from . import frame_step as fs
from .helper import gridlstm


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
        if tuple(h.shape[:2]) != (1, D) or not h.is_contiguous():
            raise ValueError("h must be one contiguous chain [1, D, H]")
        nf = n_frames.detach().cpu().numpy().astype(np.int64)
        X, Rel = fs.frame_embed(self.params, pos, vislet, n_active, F, stride=stride,
                                stream=stream)
        Xe = X.clone()                      # rows D, D+1 (vislet_emb) stay; 0..D-1 per frame
        pred = torch.zeros((S, F, 2 * fs.PRED_LEN, Nmax), device=dev)
        attn = torch.zeros((S, F, D, D), device=dev)
        cost = torch.zeros((S, F, fs.OBS_LEN, fs.OBS_LEN), device=dev)
        scratch = torch.empty((D, D), device=dev)
        c = self.cell
        h0 = h[0]                           # [D, H]: the cell reads its first 16 columns
        for s in range(S):
            for f in range(int(nf[s])):
                gridlstm(X[s, f, :D], h0, c.W, c.b, c.peep, feature_size=c.feature_size,
                         num_units=c.num_units, out=Xe[s, f, :D], state_out=scratch,
                         stream=stream)                                       # train.py:201-207
                fs.mcr_forward(self.params, Xe[s, f:f + 1], Rel[s:s + 1], G[s:s + 1],
                               n_active[s:s + 1], lam=self.lam, stream=stream,
                               out=(attn[s, f:f + 1], cost[s, f:f + 1], pred[s, f:f + 1]))
                fs.frame_recurrence(attn[s:s + 1, f:f + 1], h, stream=stream)   # :240-252
        metrics = fs.ade_fde(pred, targets, n_active, n_frames=n_frames, ped_mask=ped_mask,
                             stream=stream)                                   # :636-674
        return fs.StepOutputs(pred=pred, h=h, metrics=metrics, attn=attn, cost=cost), h
