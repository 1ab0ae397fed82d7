"""Relation operators of nri_learned.py on the GPU (C ABI).

infer_rlns(adj)      = sigmoid(adj)          (nri_learned.py:16-21)
eval_rln_ngh(adj, _) = softmax(adj, -1)      (nri_learned.py:23-28)
graph_to_kernel()    references undefined names in the reference
                     (nri_learned.py:5-13) and is not callable there either.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _as2d(adj):
    if adj.device.type != "cuda" or adj.dtype != torch.float32:
        raise ValueError("adj must be a float32 CUDA tensor (no CPU fallback)")
    a = adj.contiguous()
    cols = a.shape[-1] if a.dim() else 1
    return a, a.numel() // max(cols, 1), cols


def infer_rlns(adj_mat):
    lib = _lib.load()
    a, rows, cols = _as2d(adj_mat)
    out = torch.empty_like(a)
    _lib.check("g2k_infer_rlns_f32", lib.g2k_infer_rlns_f32(
        a.data_ptr(), out.data_ptr(), rows, cols,
        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return out


def eval_rln_ngh(adj_mat, combined_ngh=None):
    lib = _lib.load()
    a, rows, cols = _as2d(adj_mat)
    out = torch.empty_like(a)
    _lib.check("g2k_eval_rln_ngh_f32", lib.g2k_eval_rln_ngh_f32(
        a.data_ptr(), out.data_ptr(), rows, cols,
        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return out


def graph_to_kernel():
    raise NotImplementedError("nri_learned.graph_to_kernel is unimplemented in the reference "
                              "(undefined names, nri_learned.py:5-13)")
