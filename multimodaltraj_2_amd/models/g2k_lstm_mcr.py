"""g2k_lstm_mcr with the reference's constructor, attribute names and
``forward()`` (models/g2k_lstm_mcr.py:3-124); compute = g2k_mcr_forward_f32.

TF feed/fetch becomes attribute assignment: set ``outputs``, ``ngh``,
``rel_features``, ``hidden_states``, ``out_size`` (or pass ``feed=`` to
``forward``), call ``forward()``, read ``pred_path_band``, ``attn``, ``cost``.
Build decisions: Q1 the fetched prediction is the
dataflow result, never the random feed; Q2 fed tensors are used (not the
placeholder defaults); Q6 parameters are plain seeded N(0,1) tensors (the
``krnl_weights_21/*`` graph lookups are unavailable — restore trained ones
with ``weights=checkpoint_weights(prefix)``); ``sess_g`` is accepted and
ignored.  D = in_features.shape[0] in 1..16 (train.py's 16, sample.py's
num_freq_blocks = 10 and the reference checkpoints' 10).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import frame_step as fs


def _dim0(in_features):
    if isinstance(in_features, int):
        return in_features
    shape = getattr(in_features, "shape", in_features)
    return int(shape[0])


class g2k_lstm_mcr:
    def __init__(self, in_features, hidden_size, obs_len, num_nodes, lambda_reg, sess_g=None,
                 *, device="cuda", seed=0, weights=None):
        D = _dim0(in_features)
        if not 1 <= D <= fs.HIDDEN_LEN or obs_len != fs.OBS_LEN:
            raise ValueError(f"HIP g2k_lstm_mcr needs 1 <= in_features.shape[0] <= 16 and obs_len == 8 "
                             f"(got {D}, {obs_len})")
        self.D = D
        self.device = torch.device(device)
        self.out_size = int(num_nodes)
        self.lambda_reg = float(lambda_reg)
        self.hidden_size = int(hidden_size)
        rng = np.random.default_rng(seed)

        def init(shape):                         # init_w: N(0, 1) (g2k_lstm_mcr.py:10)
            return torch.from_numpy(rng.standard_normal(shape).astype(np.float32)).to(self.device)

        T, L2 = obs_len, 2 * fs.PRED_LEN
        w = weights or {}
        self.weight_v = w.get("weight_v", init((T, D + 2)))        # :49-53
        self.bias_v = w.get("bias_v", init((D,)))                  # :55-59
        self.weight_o = w.get("weight_o", init((T, self.out_size)))  # :61-64
        self.weight_c = w.get("weight_c", init((L2, T)))           # :65-69
        self.weight_r = w.get("weight_r", init((T, 2)))            # :72-76
        # placeholder_with_default feeds (:13-36, :90-94): N(0, 1) defaults
        self.outputs = init((D + 2, D))
        self.rel_features = init((2, D))
        self.visual_path = init((2, D))
        self.ngh = init((D, T))
        self.hidden_states = init((D, self.hidden_size))
        self.forward()

    def _feed(self, feed):
        for k, v in (feed or {}).items():
            name = k if isinstance(k, str) else k
            if name not in ("outputs", "ngh", "rel_features", "hidden_states", "out_size",
                            "visual_path"):
                raise KeyError(f"unknown feed {name!r}")
            if name == "out_size":
                self.out_size = int(v)
            else:
                setattr(self, name, torch.as_tensor(v, dtype=torch.float32, device=self.device))

    def forward(self, feed=None):
        """models/g2k_lstm_mcr.py:99-124 on the GPU: sets ngh (= lambda*ngh),
        attn, cost, temp_path [2L, N], pred_path_band [2, 12, N]."""
        self._feed(feed)
        n = self.out_size
        if self.weight_o.shape[1] < n:
            raise ValueError(f"weight_o has {self.weight_o.shape[1]} columns < out_size {n}")
        nmax = max(int(self.weight_o.shape[1]), 1)
        D = self.D
        params = fs.G2KParams(Wi=torch.zeros((nmax, D), device=self.device),
                              Wii=torch.zeros((D, 8), device=self.device),
                              Wv=self.weight_v.contiguous(), bv=self.bias_v.contiguous(),
                              Wr=self.weight_r.contiguous(), Wc=self.weight_c.contiguous(),
                              Wo=self.weight_o.contiguous())
        X = self.outputs.reshape(1, D + 2, D).contiguous()
        Rel = self.rel_features.reshape(1, 2, D).contiguous()
        G = self.ngh.reshape(1, D, 8).contiguous()
        nact = torch.tensor([n], dtype=torch.int32, device=self.device)
        attn, cost, pred = fs.mcr_forward(params, X, Rel, G, nact, lam=self.lambda_reg)
        self.ngh_scaled = self.lambda_reg * self.ngh
        self.attn = attn[0]
        self.cost = cost[0]
        self.temp_path = pred[0, :, :n]
        self.pred_path_band = self.temp_path.reshape(2, fs.PRED_LEN, n)
        return self.pred_path_band


def checkpoint_weights(prefix, scope_index=None, num_nodes=None, device="cuda"):
    """The g2k_lstm_mcr variables of a TF checkpoint (checkpoint.load_params:
    krnl_weights_<k>/{weight_v, bias_v, weight_o, weight_c}, krnl_embed_<k>/
    weight_r; sample.py:213-225 restores them with tf.train.Saver) as the
    ``weights=`` dict of g2k_lstm_mcr; weight_o padded with zero columns to
    ``num_nodes``."""
    from .. import checkpoint
    p = checkpoint.load_params(prefix, scope_index=scope_index, nmax=num_nodes, device=device)
    return dict(weight_v=p.Wv, bias_v=p.bv, weight_o=p.Wo, weight_c=p.Wc, weight_r=p.Wr)
