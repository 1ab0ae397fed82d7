"""Static-context input on the GPU (a5; train.py:92-113, 154-158; SURVEY.md
§8(f) row 2) through ``g2k_context_conv_f32``.

    _2dconv    = lambda * conv2d_VALID(pad(img, [[1,1],[0,1],[0,0]]), K)   [D, D]
    _2dconv_in = _2dconv @ stat_mask,  stat_mask[j][t] = t / obs_len        [D, T]

The reference draws K with an unseeded ``tf.random_normal`` of shape
[H+3-D, W+2-D, 3, 1] and reads ``ctxt.png``, which the repository does not
ship (quirk Q7): ``static_context`` takes the image as an array and a seeded
N(0, 1) filter of the reference's shape unless one is given.  The result is
the ``G`` input of the fused step.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .frame_step import HIDDEN_LEN, LAMBDA, OBS_LEN


def context_filter_shape(h: int, w: int, c: int = 3, dim: int = HIDDEN_LEN):
    """train.py:100-106: filter [width-dim+1, height-dim+1, 3] of the padded image."""
    return (h + 2 - dim + 1, w + 1 - dim + 1, c)


def static_context(img, filt=None, *, dim=HIDDEN_LEN, lam=LAMBDA, seed=0, stream=None):
    """img [H, W, C] float32 CUDA tensor -> (conv [dim, dim], G [dim, 8])."""
    lib = _lib.load()
    if not isinstance(img, torch.Tensor) or img.device.type != "cuda":
        raise ValueError("static_context runs on the GPU only (no CPU fallback)")
    if img.dim() != 3 or img.dtype != torch.float32:
        raise ValueError("img must be a float32 [H, W, C] tensor")
    img = img.contiguous()
    h, w, c = (int(x) for x in img.shape)
    shp = context_filter_shape(h, w, c, dim)
    if filt is None:
        rng = np.random.default_rng(seed)
        filt = torch.from_numpy(rng.standard_normal(shp).astype(np.float32)).to(img.device)
    if tuple(filt.shape) != shp or filt.dtype != torch.float32 or filt.device != img.device:
        raise ValueError(f"filter must be float32 {shp} on {img.device}")
    filt = filt.contiguous()
    nws = int(lib.g2k_context_conv_workspace_bytes(h, w, dim))
    if nws < 0:
        raise ValueError(f"image {h}x{w} too small for dim={dim} (dim <= 16)")
    ws = torch.empty(nws, dtype=torch.uint8, device=img.device)
    conv = torch.empty((dim, dim), dtype=torch.float32, device=img.device)
    G = torch.empty((dim, OBS_LEN), dtype=torch.float32, device=img.device)
    s = stream if stream is not None else torch.cuda.current_stream()
    rc = lib.g2k_context_conv_f32(img.data_ptr(), h, w, c, filt.data_ptr(), dim, float(lam),
                                  conv.data_ptr(), G.data_ptr(), ws.data_ptr(), nws,
                                  ctypes.c_void_p(s.cuda_stream))
    _lib.check("g2k_context_conv_f32", rc)
    return conv, G
