"""gsk_lstm_cell with the reference's constructor (models/gsk_lstm_cell.py:4-65).

The reference computes in ``__init__``: embedded = Wv @ X + bv [12, D];
cost = relu(d ngh / d ngh) = ones [12, D]; temp = (Wc [16, T] @ cost) @ Wo
[D, N]; pred = reshape(temp, (2, 12, N)).  The matmul needs T == 12 and the
reshape needs 16 N == 24 N, so at any N > 0 TensorFlow raises; this class
raises the same errors (ValueError) and produces the empty prediction for
N == 0.  No script in the reference imports it.
"""
from __future__ import annotations

import torch


class gsk_lstm_cell:
    def __init__(self, in_features, out_size, obs_len, num_nodes, lambda_reg, *, device="cuda"):
        D = int(getattr(in_features, "shape", in_features)[0]) if not isinstance(in_features, int) \
            else in_features
        self.out_size = int(num_nodes)
        self.lambda_reg = float(lambda_reg)
        wc_rows, wc_cols = 16, int(obs_len)          # weight_c [16, obs_len] (:37-41)
        cost_rows = 12                               # d ngh / d ngh has ngh's shape [12, D]
        if wc_cols != cost_rows:
            raise ValueError(f"Dimensions must be equal, but are {wc_cols} and {cost_rows} for "
                             f"MatMul (weight_c [16,{wc_cols}] @ cost [12,{D}])")
        if wc_rows * self.out_size != 2 * 12 * self.out_size:
            raise ValueError(f"Cannot reshape a tensor with {wc_rows * self.out_size} elements "
                             f"to shape [2,12,{self.out_size}] ({24 * self.out_size} elements)")
        self.pred_path_band = torch.zeros((2, 12, 0), device=device)
