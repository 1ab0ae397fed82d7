"""ctypes binding of libg2k_hip.so (the C ABI declared in include/g2k_hip.h).

The product path has no CPU fallback: if the shared library is missing or
fails to load, every entry point raises ``G2KLibraryError``.  Build it with
``python __graft_entry__.py`` (or ``make -C multimodaltraj_2_amd``).
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libg2k_hip.so")

# exported symbol -> (restype, argtypes); must match include/g2k_hip.h
c_int = ctypes.c_int
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_vp = ctypes.c_void_p


class G2KDims(ctypes.Structure):
    _fields_ = [("S", c_i32), ("F", c_i32), ("T", c_i32), ("L", c_i32), ("D", c_i32),
                ("H", c_i32), ("Nmax", c_i32), ("W", c_i32), ("stride", c_i32),
                ("flags", c_i32)]


STEP_PRED_PED_MAJOR = 1      # g2k_dims.flags (include/g2k_hip.h)
STEP_TARGETS_SHARED = 2
STEP_LOSS_NLL = 4
STEP_CORESIDENT = 8            # forward step: two workgroups per CU, launches in flight
STEP_SPLIT_SHIFT = 8           # G2K_STEP_SPLIT(x): workgroups per scene, 0 = automatic
STEP_MAX_SPLIT = 4


class G2KWeights(ctypes.Structure):
    _fields_ = [("Wi", c_vp), ("Wii", c_vp), ("Wv", c_vp), ("bv", c_vp), ("Wr", c_vp),
                ("Wc", c_vp), ("Wo", c_vp), ("head", c_vp)]


SYMBOLS = {
    "g2k_abi_version": (c_int, []),
    "g2k_last_error": (ctypes.c_char_p, []),
    "g2k_step_lds_bytes": (c_i64, [ctypes.POINTER(G2KDims)]),
    "g2k_step_workspace_bytes": (c_i64, [ctypes.POINTER(G2KDims)]),
    "g2k_step_split": (ctypes.c_int32, [ctypes.POINTER(G2KDims)]),
    "g2k_step_split_for_cus": (ctypes.c_int32, [ctypes.POINTER(G2KDims), ctypes.c_int32]),
    "g2k_workspace_init": (c_int, [c_vp, c_i64, c_vp]),
    "g2k_step_fused_f32": (c_int, [ctypes.POINTER(G2KDims), ctypes.POINTER(G2KWeights),
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_i64, c_vp]),
    "g2k_mcr_forward_f32": (c_int, [ctypes.POINTER(G2KDims), ctypes.POINTER(G2KWeights),
                                    c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp]),
    "g2k_frame_recurrence_f32": (c_int, [ctypes.POINTER(G2KDims), c_vp, c_vp, c_i32, c_vp]),
    "g2k_frame_embed_f32": (c_int, [ctypes.POINTER(G2KDims), ctypes.POINTER(G2KWeights),
                                    c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "g2k_ade_fde_f32": (c_int, [ctypes.POINTER(G2KDims), c_vp, c_vp, c_vp, c_vp, c_vp, c_i32,
                                c_vp, c_vp]),
    "g2k_infer_rlns_f32": (c_int, [c_vp, c_vp, c_i64, c_i32, c_vp]),
    "g2k_eval_rln_ngh_f32": (c_int, [c_vp, c_vp, c_i64, c_i32, c_vp]),
    "g2k_gridlstm_f32": (c_int, [c_vp, c_i64, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64,
                                 c_i32, c_i32, c_i32, c_vp]),
    "g2k_encoder_chain_f32": (c_int, [ctypes.POINTER(G2KDims), ctypes.POINTER(G2KWeights),
                                      c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i32,
                                      c_i32, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp]),
    "g2k_grad_size": (c_i64, [ctypes.POINTER(G2KDims)]),
    "g2k_grad_workspace_bytes": (c_i64, [ctypes.POINTER(G2KDims)]),
    "g2k_step_grad_f32": (c_int, [ctypes.POINTER(G2KDims), ctypes.POINTER(G2KWeights),
                                  c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp, c_vp,
                                  c_i64, c_vp]),
    "g2k_update_f32": (c_int, [c_vp, c_vp, c_vp, c_i64, c_f32, c_f32, c_f32, c_vp]),
    "g2k_nll_workspace_bytes": (c_i64, [ctypes.POINTER(G2KDims)]),
    "g2k_nll_f32": (c_int, [ctypes.POINTER(G2KDims), c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                            c_vp, c_i64, c_vp]),
    "g2k_gauss_sample_f32": (c_int, [ctypes.POINTER(G2KDims), c_vp, c_vp, ctypes.c_uint64, c_vp,
                                     c_vp]),
    "g2k_step_grad_update_f32": (c_int, [ctypes.POINTER(G2KDims), ctypes.POINTER(G2KWeights),
                                         c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_f32, c_vp,
                                         c_vp, c_i64, c_vp, c_vp, c_f32, c_f32, c_f32, c_vp]),
    "g2k_train_workspace_bytes": (c_i64, [ctypes.POINTER(G2KDims)]),
    "g2k_train_step_f32": (c_int, [ctypes.POINTER(G2KDims), ctypes.POINTER(G2KWeights),
                                   c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                                   c_vp, c_f32, c_vp, c_vp, c_i64, c_vp, c_vp, c_f32, c_f32,
                                   c_f32, c_vp]),
    "g2k_context_conv_workspace_bytes": (c_i64, [c_i32, c_i32, c_i32]),
    "g2k_context_conv_f32": (c_int, [c_vp, c_i32, c_i32, c_i32, c_vp, c_i32, c_f32, c_vp, c_vp,
                                     c_vp, c_i64, c_vp]),
    "g2k_traj_create": (c_vp, [c_vp, c_vp, c_i64, c_i32, ctypes.c_double]),
    "g2k_traj_destroy": (None, [c_vp]),
    "g2k_traj_next_step": (c_int, [c_vp, ctypes.c_double, c_i32, c_i32, c_vp, c_i32, c_vp, c_vp,
                                   c_i64, c_vp, c_vp, c_vp]),
    "g2k_traj_sample_scenes": (c_int, [c_vp, c_vp, c_i32, c_i32, c_i32, c_i32, c_i32, c_vp, c_vp,
                                       c_vp, c_vp, c_vp]),
    "g2k_scene_gather_f32": (c_int, [c_vp, c_vp, c_i64, c_vp, c_vp, c_vp, c_vp, c_i32, c_i32,
                                     c_i32, c_vp, c_vp, c_vp, c_vp, c_vp]),
}

ABI_VERSION = 9


class G2KLibraryError(RuntimeError):
    pass


class G2KError(RuntimeError):
    """A non-zero status returned across the C ABI."""

    def __init__(self, fn, code, msg):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lib = None


def load(path: str | None = None):
    """Load (once) and return the ctypes handle; raise if absent.

    torch must be imported first so that the process has exactly one HIP
    runtime (torch's bundled libamdhip64 satisfies our DT_NEEDED by soname)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise G2KLibraryError(
            f"{p} not found: the HIP library is not built (run `python __graft_entry__.py`); "
            "there is no CPU fallback")
    try:
        import torch  # noqa: F401  (one HIP runtime per process)
    except ImportError:
        pass
    try:
        lib = ctypes.CDLL(p)
    except OSError as e:
        raise G2KLibraryError(f"cannot load {p}: {e}") from e
    for name, (res, args) in SYMBOLS.items():
        fn = getattr(lib, name)  # AttributeError if a symbol is missing
        fn.restype = res
        fn.argtypes = args
    v = lib.g2k_abi_version()
    if v != ABI_VERSION:
        raise G2KLibraryError(f"ABI version mismatch: library {v}, binding {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(fn_name: str, rc: int):
    if rc != 0:
        msg = _lib.g2k_last_error().decode() if _lib is not None else "?"
        raise G2KError(fn_name, rc, msg)
