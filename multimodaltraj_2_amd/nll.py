"""The bivariate-Gaussian NLL head and its sampling path (SURVEY.md §8(f)
row 4; the reference has none, so this is the build's definition and its
parity is unpinned — see csrc/g2k_nll.hip for the formulas and
oracle/g2k_ref.py bivariate_nll / gauss_sample for the checker).

``GaussianHead`` holds the head's parameters [3, 12] (log sigma_x, log
sigma_y, atanh rho per prediction step) around the model's predictions
(pred_path_band as the fused step writes it: [S, F, 2L, Nmax]); ``nll``
returns the summed loss, the pair count, d nll / d head and (optionally)
d nll / d pred; ``sample`` draws one reproducible trajectory per
(step, pedestrian)."""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .frame_step import OBS_LEN, PRED_LEN, _check_dev, _ptr, _stream


class GaussianHead:
    def __init__(self, log_sigma=0.0, device="cuda"):
        h = torch.zeros((3, PRED_LEN), dtype=torch.float32, device=device)
        h[:2] = float(log_sigma)
        self.head = h

    def _dims(self, pred):
        S, F, L2, Nmax = (int(x) for x in pred.shape)
        if L2 != 2 * PRED_LEN:
            raise ValueError(f"pred must be [S, F, {2 * PRED_LEN}, Nmax]")
        return _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, 16, 64, Nmax, OBS_LEN, 0)

    def nll(self, pred, targets, n_active, *, n_frames=None, ped_mask=None, want_dpred=False,
            stream=None):
        """-> (nll, pairs, dhead [3, 12], dpred [S, F, 2L, Nmax] or None)."""
        lib = _lib.load()
        dev = pred.device
        d = self._dims(pred)
        S, F, Nmax = d.S, d.F, d.Nmax
        _check_dev("pred", pred, dev, torch.float32)
        _check_dev("head", self.head, dev, torch.float32)
        _check_dev("n_active", n_active, dev, torch.int32)
        if tuple(targets.shape) != (S, F, Nmax, PRED_LEN, 2):
            raise ValueError(f"targets must be [{S}, {F}, {Nmax}, {PRED_LEN}, 2]")
        _check_dev("targets", targets, dev, torch.float32)
        out = torch.empty(3 * PRED_LEN + 2, dtype=torch.float32, device=dev)
        dpred = torch.zeros_like(pred) if want_dpred else None
        ws = torch.empty(max(1, int(lib.g2k_nll_workspace_bytes(ctypes.byref(d)))), dtype=torch.uint8,
                         device=dev)
        rc = lib.g2k_nll_f32(ctypes.byref(d), _ptr(pred), _ptr(targets), _ptr(n_active),
                             _ptr(n_frames), _ptr(ped_mask), _ptr(self.head), _ptr(out), _ptr(dpred),
                             _ptr(ws), ws.numel(), _stream(stream))
        _lib.check("g2k_nll_f32", rc)
        return out[3 * PRED_LEN], out[3 * PRED_LEN + 1], out[:3 * PRED_LEN].view(3, PRED_LEN), dpred

    def sample(self, pred, seed=0, stream=None):
        """One draw around pred [S, F, 2L, Nmax] (same layout out)."""
        lib = _lib.load()
        d = self._dims(pred)
        _check_dev("pred", pred, pred.device, torch.float32)
        out = torch.empty_like(pred)
        rc = lib.g2k_gauss_sample_f32(ctypes.byref(d), _ptr(pred), _ptr(self.head),
                                      ctypes.c_uint64(int(seed)), _ptr(out), _stream(stream))
        _lib.check("g2k_gauss_sample_f32", rc)
        return out
