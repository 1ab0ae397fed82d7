"""--mode train: the reference-mode step plus a
loss, its gradient, ONE all-reduce and an optimizer update per batch.

The reference has no loss, gradient or optimizer for g2k_lstm_mcr (SURVEY.md
finding 5: its training loop re-initialises weights and fetches fed tensors);
this mode is the build's, for the north star's "RCCL all-reduce of
gradients".  loss = 1/2 the squared error of the pred_path_band rows against
the targets the ADE/FDE use; the gradient comes out of the same scene-kernel
launch as the step's outputs (g2k_train_step_f32; g2k_step_grad_f32 without
the outputs), checked against the float64 oracle ``scene_loss_grad``, itself
pinned by finite differences; unpinned against the reference, which has none.  One
flat [P + 2] buffer (gradient sums, loss, count) is all-reduced per step —
RCCL over xGMI under the nccl backend, 5.1 KB at Nmax = 32 — then every rank
applies the same update (RMSProp with global-norm clipping, argParser.py:38-47
defaults), so the replicas stay identical.  There is no CPU fallback.
"""
from __future__ import annotations

import contextlib
import ctypes

import torch
import torch.distributed as dist

from . import _lib
from .dist import allreduce_grad
from .frame_step import (HIDDEN_LEN, LAMBDA, OBS_LEN, PRED_LEN, G2KParams, StepPlan, _check_dev,
                         _ptr, _stream, plan_split, step_flags, step_frames, workspace)

GRAD_ORDER = ("Wi", "Wii", "Wv", "bv", "Wr", "Wc", "Wo")   # g2k_weights order
NLL_HEAD = 3 * PRED_LEN          # loss "nll": the head [3, L] follows Wo in the flat vector
LEARNING_RATE = 0.005    # argParser.py:43
DECAY_RATE = 0.95        # argParser.py:46 (RMSProp)
GRAD_CLIP = 10.0         # argParser.py:40


def grad_size(nmax: int, loss: str = "l2") -> int:
    """Floats in one parameter vector (g2k_grad_size): 24 * Nmax + 496
    (+ 36 for the NLL head)."""
    return 24 * int(nmax) + 496 + (NLL_HEAD if loss == "nll" else 0)


def flat_params(params: G2KParams, loss: str = "l2"):
    """Copy ``params`` into one flat device buffer in gradient layout and
    return (flat, G2KParams of views into it), so one update kernel and one
    all-reduce cover every parameter.  loss "nll": the head follows Wo
    (zeros — sigma = 1, rho = 0 — when params has none)."""
    keys = GRAD_ORDER + (("head",) if loss == "nll" else ())
    parts = []
    for k in keys:
        t = getattr(params, k)
        if t is None:
            t = torch.zeros((3, PRED_LEN), device=params.Wo.device, dtype=torch.float32)
        parts.append(t)
    flat = torch.cat([t.reshape(-1) for t in parts]).contiguous()
    views, o = {}, 0
    for k, t in zip(keys, parts):
        views[k] = flat[o:o + t.numel()].view(t.shape)
        o += t.numel()
    return flat, G2KParams(**views)


class GradPlan:
    """A validated launch of ``g2k_step_grad_f32`` bound to fixed buffers;
    ``run()`` returns grad [P + 2] = (gradient sums, loss, count)."""

    def __init__(self, params: G2KParams, pos, vislet, G, targets, n_active, *, n_frames=None,
                 ped_mask=None, stride=1, lam=LAMBDA, grad=None, stream=None,
                 targets_shared=False, frames=None, loss="l2", split=0):
        lib = _lib.load()
        dev = pos.device
        if dev.type != "cuda":
            raise ValueError("the gradient runs on the GPU only (no CPU fallback)")
        S, W, Nmax, two = pos.shape
        if two != 2:
            raise ValueError(f"pos: last dim {two}, expected 2")
        F = step_frames(targets, targets_shared, frames)
        params.check(dev)
        if params.nmax != Nmax:
            raise ValueError(f"params Nmax={params.nmax} but pos Nmax={Nmax}")
        exp = dict(pos=(S, W, Nmax, 2), vislet=(S, 2, Nmax), G=(S, HIDDEN_LEN, OBS_LEN),
                   targets=(S, 1 if targets_shared else F, Nmax, PRED_LEN, 2))
        for k, t in dict(pos=pos, vislet=vislet, G=G, targets=targets).items():
            if tuple(t.shape) != exp[k]:
                raise ValueError(f"{k}: shape {tuple(t.shape)}, expected {exp[k]}")
            _check_dev(k, t, dev, torch.float32)
        _check_dev("n_active", n_active, dev, torch.int32)
        if n_frames is not None:
            _check_dev("n_frames", n_frames, dev, torch.int32)
        if ped_mask is not None:
            _check_dev("ped_mask", ped_mask, dev, torch.uint8)
        if loss == "nll" and params.head is None:
            raise ValueError('loss "nll" needs params.head [3, 12]')
        split = plan_split(S, F, split, False, dev, stride=stride, targets_shared=targets_shared,
                           Nmax=Nmax, loss=loss)       # explicit: device-independent sizes
        d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, HIDDEN_LEN, 64, Nmax, W, stride,
                         step_flags("band", targets_shared, loss, split))
        P = int(lib.g2k_grad_size(ctypes.byref(d)))
        nws = int(lib.g2k_grad_workspace_bytes(ctypes.byref(d)))
        if P < 0 or nws < 0:
            _lib.check("g2k_grad_size", -1)
        self.P = P
        self.grad = grad if grad is not None else torch.empty(P + 2, device=dev,
                                                              dtype=torch.float32)
        self._ws = workspace(nws, dev, stream)
        w = params.abi()
        self._fn = lib.g2k_step_grad_f32
        self._fused = lib.g2k_step_grad_update_f32
        self._args = (ctypes.byref(d), ctypes.byref(w), _ptr(pos), _ptr(vislet), _ptr(G),
                      _ptr(targets), _ptr(n_active), _ptr(n_frames), _ptr(ped_mask),
                      ctypes.c_float(lam), self.grad.data_ptr(), self._ws.data_ptr(), nws,
                      _stream(stream))
        self._keep = (d, w, params, pos, vislet, G, targets, n_active, n_frames, ped_mask)

    def run(self) -> torch.Tensor:
        rc = self._fn(*self._args)
        if rc:
            _lib.check("g2k_step_grad_f32", rc)
        return self.grad

    def run_update(self, flat, ms, *, lr, decay, grad_clip) -> torch.Tensor:
        """One rank: the gradient and the update of ``flat`` (and ``ms``) in
        one call (g2k_step_grad_update_f32; the same results as ``run()`` +
        ``optimizer_update``, one launch fewer)."""
        if flat.numel() != self.P:
            raise ValueError(f"flat must have {self.P} entries")
        if ms is not None and ms.numel() != self.P:
            raise ValueError(f"ms must have {self.P} entries")
        rc = self._fused(*self._args[:-1], flat.data_ptr(),
                         None if ms is None else ms.data_ptr(), float(lr), float(decay),
                         float(grad_clip), self._args[-1])
        if rc:
            _lib.check("g2k_step_grad_update_f32", rc)
        return self.grad


def optimizer_update(flat, grad, *, lr=LEARNING_RATE, decay=DECAY_RATE, grad_clip=GRAD_CLIP,
                     ms=None, stream=None):
    """params -= step(grad[:P] / grad[P+1]) (g2k_update_f32): RMSProp when
    ``ms`` (the mean-square buffer, [P]) is given, else SGD."""
    lib = _lib.load()
    n = flat.numel()
    if grad.numel() != n + 2:
        raise ValueError(f"grad must have {n + 2} entries")
    rc = lib.g2k_update_f32(flat.data_ptr(), None if ms is None else ms.data_ptr(),
                            grad.data_ptr(), n, float(lr), float(decay), float(grad_clip),
                            _stream(stream))
    _lib.check("g2k_update_f32", rc)


class TrainPlan:
    """A validated launch of ``g2k_train_step_f32`` bound to fixed buffers:
    the fused step's outputs (pred, h, ADE/FDE sums) and the loss gradient
    [P + 2] from ONE scene-kernel launch (the producers turn each prediction
    tile's error into the gradient; nothing is recomputed), the per-scene
    gradient rows summed in a fixed order, and optionally the update."""

    def __init__(self, params: G2KParams, pos, vislet, G, targets, n_active, h, *, n_frames=None,
                 ped_mask=None, stride=1, lam=LAMBDA, out=None, grad=None, stream=None,
                 pred_layout="band", targets_shared=False, frames=None, loss="l2", split=0):
        lib = _lib.load()
        if loss == "nll" and params.head is None:
            raise ValueError('loss "nll" needs params.head [3, 12]')
        # one explicit split for the forward plan and the train launch alike
        split = plan_split(int(pos.shape[0]), step_frames(targets, targets_shared, frames), split,
                           False, pos.device, stride=stride, targets_shared=targets_shared,
                           Nmax=int(pos.shape[2]), loss=loss)
        self.fwd = StepPlan(params, pos, vislet, G, targets, n_active, h, n_frames=n_frames,
                            ped_mask=ped_mask, stride=stride, lam=lam, out=out, stream=stream,
                            pred_layout=pred_layout, targets_shared=targets_shared, frames=frames,
                            split=split)
        dev = pos.device
        S, W, Nmax, _ = pos.shape
        F, H = step_frames(targets, targets_shared, frames), int(h.shape[2])
        d = _lib.G2KDims(S, F, OBS_LEN, PRED_LEN, HIDDEN_LEN, H, Nmax, W, stride,
                         step_flags(pred_layout, targets_shared, loss, split))
        self.P = int(lib.g2k_grad_size(ctypes.byref(d)))
        nws = int(lib.g2k_train_workspace_bytes(ctypes.byref(d)))
        if self.P < 0 or nws < 0:
            _lib.check("g2k_train_workspace_bytes", -1)
        self.grad = grad if grad is not None else torch.empty(self.P + 2, device=dev,
                                                              dtype=torch.float32)
        self._ws = workspace(nws, dev, stream)
        o = self.fwd.out
        w = params.abi()
        self._fn = lib.g2k_train_step_f32
        self._head = (ctypes.byref(d), ctypes.byref(w), _ptr(pos), _ptr(vislet), _ptr(G),
                      _ptr(targets), _ptr(n_active), _ptr(n_frames), _ptr(ped_mask), _ptr(h),
                      _ptr(o.h), _ptr(o.pred), _ptr(o.metrics), ctypes.c_float(lam),
                      self.grad.data_ptr(), self._ws.data_ptr(), nws)
        self._stream = _stream(stream)
        self._keep = (d, w, params, pos, vislet, G, targets, n_active, n_frames, ped_mask, h)

    @property
    def out(self):
        return self.fwd.out

    def run(self, flat=None, ms=None, *, lr=LEARNING_RATE, decay=DECAY_RATE,
            grad_clip=GRAD_CLIP) -> torch.Tensor:
        """One call: outputs + grad; with ``flat`` also the update of the flat
        parameters (and ``ms``: RMSProp, else SGD).  Returns grad [P + 2]."""
        rc = self._fn(*self._head, None if flat is None else flat.data_ptr(),
                      None if ms is None else ms.data_ptr(), float(lr), float(decay),
                      float(grad_clip), self._stream)
        if rc:
            _lib.check("g2k_train_step_f32", rc)
        return self.grad


class TrainStep:
    """One train-mode step over fixed device buffers: the fused reference
    step (pred, h, ADE/FDE sums) and the loss gradient in one launch, the
    all-reduce of the flat gradient across ranks (when a process group is
    up), the update.  One rank: a single C call (g2k_train_step_f32 with the
    update).

    More input batches (same shapes, other buffers) can be bound with
    ``bind``; ``run(slot)`` steps on batch ``slot`` with the shared
    parameters and optimizer state.  The RMSProp mean squares start at one,
    as TF's RMSPropOptimizer initialises its "rms" slot."""

    kernel_names = "g2k_scene_kernel<GRAD> + g2k_grad_rows_kernel<update> (one rank)"

    def __init__(self, params: G2KParams, pos, vislet, G, targets, n_active, h, *,
                 lr=LEARNING_RATE, decay=DECAY_RATE, grad_clip=GRAD_CLIP, rmsprop=True,
                 n_frames=None, ped_mask=None, stride=1, lam=LAMBDA, out=None, group=None,
                 pred_layout="band", targets_shared=False, frames=None, loss="l2", split=0,
                 stream=None, collective=None):
        self.group = group
        self.world = (dist.get_world_size(group)
                      if dist.is_available() and dist.is_initialized() else 1)
        # the multi-rank structure (gradient -> all-reduce -> update); True on
        # one rank forces it (a one-rank group still issues the collective)
        self.collective = self.world > 1 if collective is None else bool(collective)
        if self.world > 1 and not self.collective:
            # each rank would apply its own shard's gradient: silent drift
            raise ValueError(f"collective=False in a {self.world}-rank group: the ranks' "
                             "gradients must be all-reduced (collective=None or True)")
        if self.collective and self.world == 1 and not (dist.is_available()
                                                        and dist.is_initialized()):
            raise ValueError("collective=True needs an initialised process group")
        self._layout = dict(pred_layout=pred_layout, targets_shared=targets_shared, frames=frames,
                            loss=loss, split=split, stream=stream)
        self.flat, self.params = flat_params(params, loss)
        self.P = self.flat.numel()
        self.ms = torch.ones_like(self.flat) if rmsprop else None
        self.lr, self.decay, self.grad_clip = lr, decay, grad_clip
        self._lam, self._stride = lam, stride
        self._slots = []
        self.bind(pos, vislet, G, targets, n_active, h, n_frames=n_frames, ped_mask=ped_mask,
                  out=out)

    def bind(self, pos, vislet, G, targets, n_active, h, *, n_frames=None, ped_mask=None,
             out=None) -> int:
        """Bind another input batch; returns its slot for ``run``."""
        self._slots.append(TrainPlan(self.params, pos, vislet, G, targets, n_active, h,
                                     n_frames=n_frames, ped_mask=ped_mask, stride=self._stride,
                                     lam=self._lam, out=out, **self._layout))
        return len(self._slots) - 1

    @property
    def out(self):
        return self._slots[0].out

    def outputs(self, slot=0):
        return self._slots[slot].out

    def run(self, slot=0) -> torch.Tensor:
        """Returns the (all-rank) [P + 2] buffer: gradient sums, loss, count."""
        plan = self._slots[slot]
        kw = dict(lr=self.lr, decay=self.decay, grad_clip=self.grad_clip)
        if not self.collective:                        # nothing to all-reduce: update in the call
            return plan.run(self.flat, self.ms, **kw)
        # gradient -> all-reduce -> update, all enqueued on the plan's stream
        # with no host wait between them: ProcessGroupNCCL orders its RCCL
        # stream after the CURRENT stream and makes the current stream wait
        # for the collective, so the collective is issued with the plan's
        # stream made current (gloo, CPU tests: a host copy inside gloo)
        s = self._layout["stream"]
        with torch.cuda.stream(s) if s is not None else contextlib.nullcontext():
            g = plan.run()
            allreduce_grad(g, self.group, force=True)
            optimizer_update(self.flat, g, ms=self.ms, stream=s, **kw)
        return g
