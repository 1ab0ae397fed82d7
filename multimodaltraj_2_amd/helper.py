"""Neighbourhood encoders of helper.py on the GPU (C ABI ``g2k_gridlstm_f32``).

The reference builds two ``tf.contrib.rnn.GridLSTMCell`` encoders
(helper.py:31-39 and 131-141); this module mirrors their classes and entry
points over device tensors.  The cell arithmetic is SURVEY.md Appendix C
(decoded from save/g2k_mcr_model_val_0.ckpt-0.meta), restated in
oracle/g2k_ref.py ``gridlstm_cell``:

    per frequency block k (feature_size inputs each, sequential in k):
      z   = [x_k, m_time_k, m_freq_{k-1}] @ W + b          W [fs + 2u, 3u]
      i   = sigmoid(z_i + wIf * c_freq_{k-1} + wIt * c_time_k)   (coupled gates)
      c_f = (1 - i) c_freq_{k-1} + i tanh(z_j);  c_t likewise from c_time_k
      o   = sigmoid(z_o + wOf * c_f + wOt * c_t)
      m_f = o tanh(c_f);  m_t = o tanh(c_t)
    out = concat_k [m_t, m_f];  new_state = concat_k [c_t, m_t]

Only the configuration the reference uses is supported
(share_time_frequency_weights=True, couple_input_forget_gates=True,
state_is_tuple=False, frequency_skip == feature_size); anything else raises
NotImplementedError, since the reference would build a different graph.
The reference's initial values come from TF's unseeded default
initializers, so they are not reproducible: W and the peepholes are seeded
Glorot-uniform here and b is zero; ``set_weights`` loads checkpoint tensors
(W_f_0_0, B_f_0, W_{I,O}_diag_freq{f,t}_0; tests/golden/ckpt_gridlstm.npz).
In the reference's train.py / sample.py the encoders' fetched outputs are
overridden by feeds, so they are off the frame loop.
There is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

SUPPORTED_UNITS = (1, 2, 4)
SUPPORTED_FEATURES = (2, 4, 8)


def _stream(stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def gridlstm(inputs, state, W, b, peep=None, *, feature_size=4, num_units=2, out=None,
             state_out=None, stream=None):
    """One GridLSTMCell step over the rows of ``inputs`` [R, K*feature_size];
    ``state`` [R, >= K*2*num_units] (leading columns read, any row pitch).
    Returns (out [R, K*2u], new_state [R, K*2u])."""
    lib = _lib.load()
    dev = inputs.device
    if dev.type != "cuda":
        raise ValueError("gridlstm runs on the GPU only (no CPU fallback)")
    u, fs = int(num_units), int(feature_size)
    named = [("inputs", inputs), ("state", state), ("W", W), ("b", b)]
    if peep is not None:
        named.append(("peep", peep))
    for k, t in named:
        if t.dtype != torch.float32 or t.device != dev:
            raise TypeError(f"{k}: expected float32 on {dev}")
    if inputs.dim() != 2 or inputs.stride(1) != 1:
        raise ValueError("inputs must be 2-D with unit column stride")
    if state.dim() != 2 or state.stride(1) != 1:
        raise ValueError("state must be 2-D with unit column stride")
    R, ncol = int(inputs.shape[0]), int(inputs.shape[1])
    if ncol % fs:
        raise ValueError(f"inputs has {ncol} columns, not a multiple of feature_size={fs}")
    K = ncol // fs
    if int(state.shape[0]) != R or int(state.shape[1]) < 2 * u * K:
        raise ValueError(f"state must be [{R}, >= {2 * u * K}], got {tuple(state.shape)}")
    if tuple(W.shape) != (fs + 2 * u, 3 * u) or tuple(b.shape) != (3 * u,):
        raise ValueError(f"W must be [{fs + 2 * u}, {3 * u}] and b [{3 * u}]")
    if peep is not None and tuple(peep.shape) != (4, u):
        raise ValueError(f"peep must be [4, {u}] (wIf, wIt, wOf, wOt)")
    W, b = W.contiguous(), b.contiguous()
    peep = peep.contiguous() if peep is not None else None
    if out is None:
        out = torch.empty((R, 2 * u * K), device=dev, dtype=torch.float32)
    if state_out is None:
        state_out = torch.empty((R, 2 * u * K), device=dev, dtype=torch.float32)
    rc = lib.g2k_gridlstm_f32(inputs.data_ptr(), inputs.stride(0), state.data_ptr(),
                              state.stride(0), W.data_ptr(), b.data_ptr(),
                              None if peep is None else peep.data_ptr(), out.data_ptr(),
                              state_out.data_ptr(), R, K, fs, u, _stream(stream))
    _lib.check("g2k_gridlstm_f32", rc)
    return out, state_out


def _glorot(rng, shape):
    fan_in, fan_out = shape[0], shape[-1]
    lim = np.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=shape).astype(np.float32)


class GridLSTMCell:
    """Mirror of tf.contrib.rnn.GridLSTMCell as helper.py configures it."""

    def __init__(self, num_units, feature_size, frequency_skip, use_peepholes,
                 num_frequency_blocks, share_time_frequency_weights=True, state_is_tuple=False,
                 couple_input_forget_gates=True, reuse=None, seed=0, device=None):
        if not share_time_frequency_weights or not couple_input_forget_gates or state_is_tuple:
            raise NotImplementedError("only the helper.py configuration is supported "
                                      "(shared weights, coupled gates, concatenated state)")
        if frequency_skip != feature_size:
            raise NotImplementedError("frequency_skip must equal feature_size (helper.py:33)")
        if num_units not in SUPPORTED_UNITS or feature_size not in SUPPORTED_FEATURES:
            raise NotImplementedError(f"num_units in {SUPPORTED_UNITS}, feature_size in "
                                      f"{SUPPORTED_FEATURES}")
        self.num_units = int(num_units)
        self.feature_size = int(feature_size)
        self.num_frequency_blocks = [int(n) for n in num_frequency_blocks]
        self.use_peepholes = bool(use_peepholes)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        rng = np.random.default_rng(seed)
        u, fs = self.num_units, self.feature_size
        self.W = torch.from_numpy(_glorot(rng, (fs + 2 * u, 3 * u))).to(self.device)
        self.b = torch.zeros(3 * u, dtype=torch.float32, device=self.device)
        self.peep = (torch.from_numpy(_glorot(rng, (4, u))).to(self.device)
                     if self.use_peepholes else None)

    @property
    def output_size(self) -> int:
        return 2 * self.num_units * sum(self.num_frequency_blocks)

    @property
    def state_size(self) -> int:
        return 2 * self.num_units * sum(self.num_frequency_blocks)

    def set_weights(self, W, b, peep=None):
        """Load W [fs+2u, 3u], b [3u] and (with peepholes) peep [4, u] =
        (wIf, wIt, wOf, wOt), e.g. from a reference checkpoint."""
        u, fs = self.num_units, self.feature_size
        W = torch.as_tensor(np.asarray(W, dtype=np.float32)).to(self.device)
        b = torch.as_tensor(np.asarray(b, dtype=np.float32)).to(self.device)
        if tuple(W.shape) != (fs + 2 * u, 3 * u) or tuple(b.shape) != (3 * u,):
            raise ValueError("weight shapes do not match the cell")
        self.W, self.b = W.contiguous(), b.contiguous()
        if self.use_peepholes:
            if peep is None:
                raise ValueError("this cell uses peepholes: peep [4, u] is required")
            p = torch.as_tensor(np.asarray(peep, dtype=np.float32)).to(self.device)
            if tuple(p.shape) != (4, u):
                raise ValueError("peep must be [4, u]")
            self.peep = p.contiguous()

    def share_weights_with(self, other: "GridLSTMCell"):
        """reuse=True in the reference (helper.py:139): the static encoder's
        cell reads the vis/loc encoder's W_f_0_0 / B_f_0."""
        if (other.num_units, other.feature_size) != (self.num_units, self.feature_size):
            raise ValueError("cells differ in num_units / feature_size")
        self.W, self.b = other.W, other.b

    def __call__(self, inputs, state, stream=None):
        # tf.contrib GridLSTMCell slices block f from columns [f * skip, f * skip +
        # feature_size) and requires int((ncol - feature_size) / skip) + 1 blocks:
        # a 10-column input (sample.py's num_freq_blocks = 10) feeds 2 blocks of
        # 4 and its last 2 columns are never read
        K = sum(self.num_frequency_blocks)
        ncol = int(inputs.shape[1])
        if ncol < self.feature_size or (ncol - self.feature_size) // self.feature_size + 1 != K:
            raise ValueError(f"inputs with {ncol} columns do not make {K} blocks of {self.feature_size}")
        inputs = inputs[:, :K * self.feature_size]
        return gridlstm(inputs, state, self.W, self.b, self.peep,
                        feature_size=self.feature_size, num_units=self.num_units, stream=stream)


class neighborhood_vis_loc_encoder:
    """helper.py:10-75: GridLSTM over the [hidden_len, hidden_len] frame input
    with peepholes; ``forward`` sets ``output`` and ``c_hidden_state``."""

    def __init__(self, hidden_size, hidden_len, num_layers, grid_size, embedding_size,
                 dropout=0, device=None, seed=0):
        self.hidden_size = hidden_size
        self.embedding_size = embedding_size
        self.hidden_len = hidden_len
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.rnn = GridLSTMCell(num_units=num_layers, feature_size=grid_size,
                                frequency_skip=grid_size, use_peepholes=True,
                                num_frequency_blocks=[int(hidden_len / grid_size)],
                                share_time_frequency_weights=True, state_is_tuple=False,
                                couple_input_forget_gates=True, seed=seed, device=self.device)
        self.input = torch.zeros((hidden_len, hidden_len), dtype=torch.float32, device=self.device)
        self.state_f00_b00_c = torch.zeros((hidden_len, hidden_size), dtype=torch.float32,
                                           device=self.device)
        self.output = None
        self.c_hidden_state = None

    def update_input_size(self, new_size):
        """helper.py:57-59: re-shape the input / state feeds."""
        self.input = torch.zeros((new_size, new_size), dtype=torch.float32, device=self.device)
        self.hidden_state = torch.zeros((new_size, self.hidden_size), dtype=torch.float32,
                                        device=self.device)

    def forward(self, inputs=None, state=None, stream=None):
        """helper.py:61-68: output, c_hidden_state = rnn(inputs, state)."""
        if inputs is not None:
            self.input = inputs
        if state is not None:
            self.state_f00_b00_c = state
        self.output, self.c_hidden_state = self.rnn(self.input, self.state_f00_b00_c, stream)
        return self.output, self.c_hidden_state

    def init_hidden(self, size):
        """helper.py:74-75."""
        return torch.zeros((size, self.hidden_size), dtype=torch.float32, device=self.device)


class neighborhood_stat_enc:
    """helper.py:77-141: GridLSTM over the static-context input [dim, 8]
    without peepholes, grid_size/2 frequency blocks.  ``ctxt_path`` is kept
    for signature parity (the reference's image load is commented out);
    ``share_with`` reproduces its reuse of the vis/loc encoder's weights."""

    def __init__(self, ctxt_path, hidden_size, num_layers, grid_size, dim, device=None, seed=1,
                 share_with: neighborhood_vis_loc_encoder | None = None):
        self.ctxt_path = ctxt_path
        self.hidden_size = hidden_size
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.rnn = GridLSTMCell(num_units=num_layers, feature_size=grid_size,
                                frequency_skip=grid_size, use_peepholes=False,
                                num_frequency_blocks=[int(grid_size / 2)],
                                share_time_frequency_weights=True, state_is_tuple=False,
                                couple_input_forget_gates=True, reuse=True, seed=seed,
                                device=self.device)
        if share_with is not None:
            self.rnn.share_weights_with(share_with.rnn)
        self.input = torch.zeros((dim, 8), dtype=torch.float32, device=self.device)
        self.hidden_state = torch.zeros((dim, hidden_size), dtype=torch.float32, device=self.device)
        self.output = None
        self.c_hidden_states = None

    def forward(self, inputs=None, state=None, stream=None):
        """helper.py:141: output, c_hidden_states = rnn(input, hidden_state)."""
        if inputs is not None:
            self.input = inputs
        if state is not None:
            self.hidden_state = state
        self.output, self.c_hidden_states = self.rnn(self.input, self.hidden_state, stream)
        return self.output, self.c_hidden_states
