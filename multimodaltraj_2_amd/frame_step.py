"""Host API of the fused per-frame step (train.py:197-276) over device tensors.

Everything here is plumbing around the C ABI (include/g2k_hip.h): it checks
shapes/dtypes/devices on the host, allocates outputs with torch, and calls
``g2k_step_fused_f32`` / ``g2k_mcr_forward_f32`` / ``g2k_frame_recurrence_f32``
/ ``g2k_ade_fde_f32`` on the current HIP stream.  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, fields

import numpy as np
import torch

from . import _lib

OBS_LEN = 8          # argParser.py:26-28
PRED_LEN = 12        # models/g2k_lstm_mcr.py:124 hard-codes 12
HIDDEN_LEN = 16      # neighborhood_size / grid_size = 64 / 4 (train.py:93)
LAMBDA = 5e-4        # argParser.py --lambda_param
METRIC_FIELDS = ("ade_spec_sum", "count", "fde_sq_sum", "ade_l2_sum", "fde_l2_sum",
                 "frames", "reserved0", "reserved1")


@dataclass
class G2KParams:
    """Model parameters, shapes as in the reference (padded to Nmax where the
    reference sizes them by the batch's num_nodes)."""
    Wi: torch.Tensor    # [Nmax, D]   train.py:168-171
    Wii: torch.Tensor   # [D, T]      train.py:172-175
    Wv: torch.Tensor    # [T, D+2]    models/g2k_lstm_mcr.py:49-53
    bv: torch.Tensor    # [D]         models/g2k_lstm_mcr.py:55-59
    Wr: torch.Tensor    # [T, 2]      models/g2k_lstm_mcr.py:72-76
    Wc: torch.Tensor    # [2L, T]     models/g2k_lstm_mcr.py:65-69
    Wo: torch.Tensor    # [T, Nmax]   models/g2k_lstm_mcr.py:61-64
    head: torch.Tensor | None = None   # [3, L] NLL head (train mode, loss "nll"; the build's)

    @property
    def nmax(self) -> int:
        return int(self.Wi.shape[0])

    def to(self, device) -> "G2KParams":
        return G2KParams(**{f.name: (None if getattr(self, f.name) is None
                                     else getattr(self, f.name).to(device)) for f in fields(self)})

    def numpy(self) -> dict:
        return {f.name: getattr(self, f.name).detach().cpu().numpy() for f in fields(self)
                if getattr(self, f.name) is not None}

    def check(self, device):
        D, T, L2 = HIDDEN_LEN, OBS_LEN, 2 * PRED_LEN
        n = self.nmax
        want = dict(Wi=(n, D), Wii=(D, T), Wv=(T, D + 2), bv=(D,), Wr=(T, 2), Wc=(L2, T),
                    Wo=(T, n))
        if self.head is not None:
            want["head"] = (3, PRED_LEN)
        for k, shp in want.items():
            t = getattr(self, k)
            if tuple(t.shape) != shp:
                raise ValueError(f"param {k}: shape {tuple(t.shape)}, expected {shp}")
            _check_dev(k, t, device, torch.float32)

    def abi(self) -> _lib.G2KWeights:
        return _lib.G2KWeights(*(None if getattr(self, f.name) is None else
                                 getattr(self, f.name).data_ptr() for f in fields(self)))


def init_params(nmax: int, seed: int = 0, device="cpu") -> G2KParams:
    """~N(0, 1) weights (init_w stddev 1, train.py:116-117 /
    models/g2k_lstm_mcr.py:10), generated on the host with a seeded NumPy
    Generator so the oracle sees the same values."""
    rng = np.random.default_rng(seed)
    D, T, L2 = HIDDEN_LEN, OBS_LEN, 2 * PRED_LEN
    shapes = [("Wi", (nmax, D)), ("Wii", (D, T)), ("Wv", (T, D + 2)), ("bv", (D,)),
              ("Wr", (T, 2)), ("Wc", (L2, T)), ("Wo", (T, nmax))]
    return G2KParams(**{k: torch.from_numpy(rng.standard_normal(s).astype(np.float32)).to(device)
                        for k, s in shapes})


def _check_dev(name, t, device, dtype):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name}: expected a torch.Tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: dtype {t.dtype}, expected {dtype}")
    if t.device != device:
        raise ValueError(f"{name}: on {t.device}, expected {device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def _ptr(t):
    return None if t is None else t.data_ptr()


def _stream(stream):
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def step_flags(pred_layout="band", targets_shared=False, loss="l2", split=0,
               coresident=False) -> int:
    """g2k_dims.flags: pred_layout "band" = pred_path_band [S, F, 2L, Nmax],
    "ped" = pedestrian-major [S, F, Nmax, L, 2]; targets_shared = one
    [S, 1, Nmax, L, 2] target set for every frame; loss (train mode) "l2" =
    1/2 the squared error, "nll" = the bivariate-Gaussian NLL (params.head);
    split = workgroups per scene (0: automatic, G2K_STEP_SPLIT); coresident
    (forward step only) = the caller keeps launches in flight on several
    streams: two 8-wave workgroups per CU (G2K_STEP_CORESIDENT)."""
    if pred_layout not in ("band", "ped"):
        raise ValueError(f"pred_layout {pred_layout!r}: 'band' or 'ped'")
    if loss not in ("l2", "nll"):
        raise ValueError(f"loss {loss!r}: 'l2' or 'nll'")
    if not 0 <= int(split) <= _lib.STEP_MAX_SPLIT:
        raise ValueError(f"split {split}: 0 (automatic) .. {_lib.STEP_MAX_SPLIT}")
    return ((_lib.STEP_PRED_PED_MAJOR if pred_layout == "ped" else 0)
            | (_lib.STEP_TARGETS_SHARED if targets_shared else 0)
            | (_lib.STEP_LOSS_NLL if loss == "nll" else 0)
            | (_lib.STEP_CORESIDENT if coresident else 0)
            | (int(split) << _lib.STEP_SPLIT_SHIFT))


def pred_shape(S, F, Nmax, pred_layout="band"):
    return (S, F, 2 * PRED_LEN, Nmax) if pred_layout == "band" else (S, F, Nmax, PRED_LEN, 2)


def pred_band(pred, pred_layout="band"):
    """Either layout -> pred_path_band [S, F, 2L, Nmax] (a view or a copy)."""
    if pred_layout == "band":
        return pred
    S, F, N = pred.shape[:3]
    return pred.permute(0, 1, 4, 3, 2).reshape(S, F, 2 * PRED_LEN, N)


@dataclass
class StepOutputs:
    pred: torch.Tensor       # [S, F, 2L, Nmax] (pred_layout "ped": [S, F, Nmax, L, 2])
    h: torch.Tensor          # [S, D, H]
    metrics: torch.Tensor    # [S, 8]
    attn: torch.Tensor | None = None   # [S, F, D, D]
    cost: torch.Tensor | None = None   # [S, F, T, T]


def step_lds_bytes(S, F, H, Nmax, W, stride, coresident=False, targets_shared=False) -> int:
    lib = _lib.load()
    d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, HIDDEN_LEN, H, Nmax, W, stride,
                     step_flags(coresident=coresident, targets_shared=targets_shared))
    return int(lib.g2k_step_lds_bytes(ctypes.byref(d)))


CORESIDENT_LDS = 80 * 1024     # g2k_scene.hip kCoresidentLds


def step_coresidency(S, F, H, Nmax, W, stride, coresident=False, targets_shared=False) -> int:
    """Workgroups of one step launch a CU holds at once: 2 under
    G2K_STEP_CORESIDENT when the 8-wave geometry applies (H < 512 and the
    scene's LDS fits twice, include/g2k_hip.h), else 1."""
    if not coresident or H >= 512:
        return 1
    lds = step_lds_bytes(S, F, H, Nmax, W, stride, True, targets_shared)
    return 2 if lds <= CORESIDENT_LDS else 1


def device_cus(device) -> int:
    """Compute units of the device a plan will launch on."""
    return int(torch.cuda.get_device_properties(device).multi_processor_count)


def split_for_cus(S, F, split=0, coresident=False, cus=256, *, stride=1, targets_shared=False,
                  Nmax=1, loss="l2") -> int:
    """Workgroups per scene for a device with ``cus`` CUs: the request, or the
    library's automatic choice (g2k_step_split_for_cus, ABI 9: host
    arithmetic, no HIP call — the same answer with or without a GPU).  The
    choice is 1 for loop-invariant launches (stride 0 with shared targets:
    one frame's work per chunk, g2k_scene.hip frames_invariant), so the
    stride, the targets' sharing, Nmax and the loss take part."""
    lib = _lib.load()
    W = (max(F, 1) - 1) * stride + OBS_LEN
    d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, HIDDEN_LEN, 128, max(int(Nmax), 1), W, stride,
                     step_flags(targets_shared=targets_shared, loss=loss, split=split,
                                coresident=coresident))
    x = int(lib.g2k_step_split_for_cus(ctypes.byref(d), int(cus)))
    if x < 1:
        _lib.check("g2k_step_split_for_cus", -1)
    return x


def plan_split(S, F, split, coresident, device, **kw) -> int:
    """The explicit split a plan launches with: an automatic request (0) is
    resolved HERE for the plan's own device and passed to the library as
    G2K_STEP_SPLIT(x), so sizing and launch never depend on which device is
    current (include/g2k_hip.h); 0 stays 0 under G2K_STEP_CORESIDENT (the
    library's 1).  ``kw``: split_for_cus's stride / targets_shared / Nmax /
    loss."""
    if split or coresident:
        return split
    return split_for_cus(S, F, 0, False, device_cus(device), **kw)


def step_split(S, F, H, Nmax, W, stride, split=0, coresident=False, device=None,
               targets_shared=False) -> int:
    """Workgroups per scene a plan on ``device`` (default: the current one)
    uses: the request, or the automatic choice for that device's CUs."""
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    return split_for_cus(S, F, split, coresident, device_cus(dev), stride=stride,
                         targets_shared=targets_shared, Nmax=Nmax)


def step_workspace_bytes(S, F, H, Nmax, W, stride) -> int:
    lib = _lib.load()
    d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, HIDDEN_LEN, H, Nmax, W, stride)
    return int(lib.g2k_step_workspace_bytes(ctypes.byref(d)))


def workspace(nbytes, device, stream=None):
    """A launch plan's own workspace, zero-filled ON THE PLAN'S STREAM (split
    scenes keep per-scene tickets in it that every call leaves at zero, so the
    first fill must be stream-ordered before the first launch, which may run
    on a stream other than the current one; include/g2k_hip.h)."""
    s = stream if stream is not None else torch.cuda.current_stream(device)
    with torch.cuda.stream(s):
        return torch.zeros(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def step_fused(params: G2KParams, pos, vislet, G, targets, n_active, h, *, n_frames=None,
               ped_mask=None, stride=1, lam=LAMBDA, out: StepOutputs | None = None,
               want_attn=False, stream=None, h_out=None, pred_layout="band",
               targets_shared=False, frames=None, split=0, coresident=False) -> StepOutputs:
    """One pass of the per-frame body of train.py:197-276 over S scenes.

    pos [S, W, Nmax, 2], vislet [S, 2, Nmax], G [S, D, T],
    targets [S, F, Nmax, L, 2] (targets_shared: [S, 1, Nmax, L, 2] and F =
    ``frames``), n_active [S] int32, h [S, D, H].  ``F`` is taken from
    ``targets`` otherwise.  Returns pred (``pred_layout``, see step_flags) /
    h / metrics (and per-frame attn / cost when ``want_attn``)."""
    plan = StepPlan(params, pos, vislet, G, targets, n_active, h, n_frames=n_frames,
                    ped_mask=ped_mask, stride=stride, lam=lam, out=out, want_attn=want_attn,
                    stream=stream, h_out=h_out, pred_layout=pred_layout,
                    targets_shared=targets_shared, frames=frames, split=split,
                    coresident=coresident)
    plan.run()
    return plan.out


class StepPlan:
    """A validated launch of ``g2k_step_fused_f32`` bound to fixed device
    buffers: the checks, the output allocation and the C argument list are
    built once; ``run()`` is a single call across the C ABI on the bound
    stream.  The buffers' contents may change between runs (that is how a
    training loop feeds the next batch); their shapes and addresses may not."""

    def __init__(self, params: G2KParams, pos, vislet, G, targets, n_active, h, *,
                 n_frames=None, ped_mask=None, stride=1, lam=LAMBDA,
                 out: StepOutputs | None = None, want_attn=False, stream=None, h_out=None,
                 pred_layout="band", targets_shared=False, frames=None, split=0,
                 coresident=False):
        self._fn, self._args, self.out, self._keep = _prepare_step(
            params, pos, vislet, G, targets, n_active, h, n_frames, ped_mask, stride, lam, out,
            want_attn, stream, h_out, pred_layout, targets_shared, frames, split, coresident)

    def run(self) -> StepOutputs:
        rc = self._fn(*self._args)
        if rc:
            _lib.check("g2k_step_fused_f32", rc)
        return self.out


def step_frames(targets, targets_shared, frames):
    """F of a step: targets.shape[1], or ``frames`` with shared targets."""
    if not targets_shared:
        return int(targets.shape[1])
    if frames is None:
        raise ValueError("targets_shared needs frames (F)")
    return int(frames)


def _prepare_step(params, pos, vislet, G, targets, n_active, h, n_frames, ped_mask, stride, lam,
                  out, want_attn, stream, h_out, pred_layout="band", targets_shared=False,
                  frames=None, split=0, coresident=False):
    lib = _lib.load()
    dev = pos.device
    if dev.type != "cuda":
        raise ValueError("step_fused runs on the GPU only (no CPU fallback)")
    S, W, Nmax, two = pos.shape
    if two != 2:
        raise ValueError(f"pos: last dim {two}, expected 2")
    F = step_frames(targets, targets_shared, frames)
    split = plan_split(S, F, split, coresident, dev, stride=stride, targets_shared=targets_shared,
                       Nmax=Nmax)
    flags = step_flags(pred_layout, targets_shared, split=split, coresident=coresident)
    H = int(h.shape[2])
    params.check(dev)
    if params.nmax != Nmax:
        raise ValueError(f"params Nmax={params.nmax} but pos Nmax={Nmax}")
    exp = dict(pos=(S, W, Nmax, 2), vislet=(S, 2, Nmax), G=(S, HIDDEN_LEN, OBS_LEN),
               targets=(S, 1 if targets_shared else F, Nmax, PRED_LEN, 2), h=(S, HIDDEN_LEN, H))
    for k, t in dict(pos=pos, vislet=vislet, G=G, targets=targets, h=h).items():
        if tuple(t.shape) != exp[k]:
            raise ValueError(f"{k}: shape {tuple(t.shape)}, expected {exp[k]}")
        _check_dev(k, t, dev, torch.float32)
    if tuple(n_active.shape) != (S,):
        raise ValueError("n_active must be [S]")
    _check_dev("n_active", n_active, dev, torch.int32)
    if n_frames is not None:
        _check_dev("n_frames", n_frames, dev, torch.int32)
    if ped_mask is not None:
        _check_dev("ped_mask", ped_mask, dev, torch.uint8)
        if tuple(ped_mask.shape) != (S, Nmax):
            raise ValueError("ped_mask must be [S, Nmax]")
    if out is None:
        # the kernel writes pred for frames < n_frames and columns < n_active
        # only: the rest stays as allocated (zero)
        out = StepOutputs(
            pred=torch.zeros(pred_shape(S, F, Nmax, pred_layout), device=dev, dtype=torch.float32),
            h=h_out if h_out is not None else torch.empty_like(h),
            metrics=torch.empty((S, 8), device=dev, dtype=torch.float32),
            attn=(torch.empty((S, F, HIDDEN_LEN, HIDDEN_LEN), device=dev, dtype=torch.float32)
                  if want_attn else None),
            cost=(torch.empty((S, F, OBS_LEN, OBS_LEN), device=dev, dtype=torch.float32)
                  if want_attn else None))
    if tuple(out.pred.shape) != pred_shape(S, F, Nmax, pred_layout):
        raise ValueError(f"out.pred: shape {tuple(out.pred.shape)}, expected "
                         f"{pred_shape(S, F, Nmax, pred_layout)} ({pred_layout})")
    d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, HIDDEN_LEN, H, Nmax, W, stride, flags)
    w = params.abi()
    nws = int(lib.g2k_step_workspace_bytes(ctypes.byref(d)))
    if nws < 0:
        _lib.check("g2k_step_workspace_bytes", -1)
    ws = workspace(nws, dev, stream)
    args = (ctypes.byref(d), ctypes.byref(w), _ptr(pos), _ptr(vislet), _ptr(G), _ptr(targets),
            _ptr(n_active), _ptr(n_frames), _ptr(ped_mask), _ptr(h), _ptr(out.h), _ptr(out.pred),
            _ptr(out.metrics), _ptr(out.attn), _ptr(out.cost), ctypes.c_float(lam),
            ws.data_ptr(), nws, _stream(stream))
    # keep the tensors and ctypes structs the pointers refer to alive
    keep = (d, w, params, pos, vislet, G, targets, n_active, n_frames, ped_mask, h, ws)
    return lib.g2k_step_fused_f32, args, out, keep


def frame_embed(params: G2KParams, pos, vislet, n_active, F, *, stride=1, X=None, Rel=None,
                stream=None):
    """The model input of every frame (g2k_frame_embed_f32; train.py:76-85,
    167-195): pos [S, W, Nmax, 2], vislet [S, 2, Nmax] -> X [S, F, D+2, D]
    ([Wii @ (B_f @ Wi); vislet @ Wi] of frame f's window rows f*stride + t)
    and Rel [S, 2, D] = (vislet @ Wi)^2."""
    lib = _lib.load()
    dev = pos.device
    S, W, Nmax, _ = pos.shape
    _check_dev("pos", pos, dev, torch.float32)
    _check_dev("vislet", vislet, dev, torch.float32)
    _check_dev("n_active", n_active, dev, torch.int32)
    params.check(dev)
    if tuple(vislet.shape) != (S, 2, Nmax) or params.nmax != Nmax:
        raise ValueError("vislet must be [S, 2, Nmax] and params Nmax must match pos")
    D = HIDDEN_LEN
    X = X if X is not None else torch.empty((S, F, D + 2, D), device=dev, dtype=torch.float32)
    Rel = Rel if Rel is not None else torch.empty((S, 2, D), device=dev, dtype=torch.float32)
    if tuple(X.shape) != (S, F, D + 2, D) or tuple(Rel.shape) != (S, 2, D):
        raise ValueError("X must be [S, F, D+2, D] and Rel [S, 2, D]")
    d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, D, 64, Nmax, W, stride)
    w = params.abi()
    rc = lib.g2k_frame_embed_f32(ctypes.byref(d), ctypes.byref(w), _ptr(pos), _ptr(vislet),
                                 _ptr(n_active), _ptr(X), _ptr(Rel), _stream(stream))
    _lib.check("g2k_frame_embed_f32", rc)
    return X, Rel


def mcr_forward(params: G2KParams, X, Rel, G, n_active, *, lam=LAMBDA, stream=None, out=None):
    """g2k_lstm_mcr.forward() for S feeds (models/g2k_lstm_mcr.py:99-124).
    X [S, D+2, D], Rel [S, 2, D], G [S, D, T] -> (attn [S,D,D], cost [S,T,T],
    pred [S, 2L, Nmax]); D = X.shape[2] in 1..16 (sample.py runs D = 10,
    the reference checkpoints hold D = 10 weights).  ``out``: (attn, cost,
    pred) tensors of those shapes to write into (contiguous views allowed)."""
    lib = _lib.load()
    dev = X.device
    S = int(X.shape[0])
    D = int(X.shape[2]) if X.dim() == 3 else -1
    Nmax = int(params.Wo.shape[1])
    for k, t, shp in (("X", X, (S, D + 2, D)), ("Rel", Rel, (S, 2, D)), ("G", G, (S, D, OBS_LEN)),
                      ("Wv", params.Wv, (OBS_LEN, D + 2)), ("bv", params.bv, (D,))):
        if tuple(t.shape) != shp:
            raise ValueError(f"{k}: shape {tuple(t.shape)}, expected {shp}")
        _check_dev(k, t, dev, torch.float32)
    _check_dev("n_active", n_active, dev, torch.int32)
    for k in ("Wr", "Wc", "Wo"):
        _check_dev(k, getattr(params, k), dev, torch.float32)
    if out is None:
        attn = torch.empty((S, D, D), device=dev, dtype=torch.float32)
        cost = torch.empty((S, OBS_LEN, OBS_LEN), device=dev, dtype=torch.float32)
        pred = torch.empty((S, 2 * PRED_LEN, Nmax), device=dev, dtype=torch.float32)
    else:
        attn, cost, pred = out
        for k, t, shp in (("attn", attn, (S, D, D)), ("cost", cost, (S, OBS_LEN, OBS_LEN)),
                          ("pred", pred, (S, 2 * PRED_LEN, Nmax))):
            if tuple(t.shape) != shp:
                raise ValueError(f"out {k}: shape {tuple(t.shape)}, expected {shp}")
            _check_dev(k, t, dev, torch.float32)
    d = _lib.G2KDims(S, 1, OBS_LEN, PRED_LEN, D, 64, Nmax, OBS_LEN, 0)
    w = _lib.G2KWeights(None, None, params.Wv.data_ptr(), params.bv.data_ptr(),
                        params.Wr.data_ptr(), params.Wc.data_ptr(), params.Wo.data_ptr())
    rc = lib.g2k_mcr_forward_f32(ctypes.byref(d), ctypes.byref(w), _ptr(X), _ptr(Rel), _ptr(G),
                                 _ptr(n_active), _ptr(attn), _ptr(cost), _ptr(pred), float(lam),
                                 _stream(stream))
    _lib.check("g2k_mcr_forward_f32", rc)
    return attn, cost, pred


def frame_recurrence(A, h, *, stream=None):
    """train.py:240-252 over F attention matrices: A [S, F, D, D], h [S, D, H]
    (updated in place and returned); D in 1..16."""
    lib = _lib.load()
    S, F = int(A.shape[0]), int(A.shape[1])
    H = int(h.shape[2])
    D = int(h.shape[1])
    _check_dev("A", A, A.device, torch.float32)
    _check_dev("h", h, A.device, torch.float32)
    if tuple(A.shape[2:]) != (D, D) or tuple(h.shape) != (S, D, H):
        raise ValueError(f"A must be [S, F, D, D] and h [S, D, H] (got {tuple(A.shape)}, {tuple(h.shape)})")
    d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, D, H, 1, OBS_LEN, 0)
    rc = lib.g2k_frame_recurrence_f32(ctypes.byref(d), _ptr(A), _ptr(h), F, _stream(stream))
    _lib.check("g2k_frame_recurrence_f32", rc)
    return h


def ade_fde(pred, targets, n_active, *, n_frames=None, ped_mask=None, variant=0,
            obs_length=OBS_LEN, stream=None):
    """Error sums from predictions.  variant 0: train.py:640-674 sums
    (pred [S, F, 2L, Nmax], targets [S, F, Nmax, L, 2]); variant 1:
    sample.py get_mean_error (pred [S, 2L, Nmax], targets [S, Nmax, L, 2]).
    Returns [S, 8]."""
    lib = _lib.load()
    dev = pred.device
    if variant == 0:
        S, F, _, Nmax = pred.shape
    else:
        S, _, Nmax = pred.shape
        F = 1
    out = torch.empty((S, 8), device=dev, dtype=torch.float32)
    T = OBS_LEN if variant == 0 else obs_length
    d = _lib.G2KDims(S, F, T, PRED_LEN, HIDDEN_LEN, 64, Nmax, OBS_LEN, 0)
    if variant == 1:
        # the kernel reads obs_length from d.T; geometry checks need T=8, so
        # only the default observed length is accepted here
        if obs_length != OBS_LEN:
            raise ValueError("get_mean_error variant supports observed_length=8 only")
    for k, t in (("pred", pred), ("targets", targets)):
        _check_dev(k, t, dev, torch.float32)
    rc = lib.g2k_ade_fde_f32(ctypes.byref(d), _ptr(pred), _ptr(targets), _ptr(n_active),
                             _ptr(n_frames), _ptr(ped_mask), int(variant), _ptr(out),
                             _stream(stream))
    _lib.check("g2k_ade_fde_f32", rc)
    return out


def batch_errors(metrics: torch.Tensor, leave_dataset=None, num_nodes=None):
    """train.py:668-674 per-batch reduction of the metric sums -> (ADE_b, FDE_b)
    per scene, on the host."""
    m = metrics.detach().double().cpu().numpy()
    ade = np.where(m[:, 1] > 0, m[:, 0] / np.maximum(m[:, 1], 1), np.nan)
    denom = np.asarray(num_nodes, dtype=np.float64) if leave_dataset == 5 else m[:, 5]
    fde = np.where(m[:, 1] > 0, np.sqrt(m[:, 2]) / np.maximum(denom, 1), np.nan)
    return ade, fde
