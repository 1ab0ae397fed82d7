"""Synthetic ETH-shaped scene batches (SURVEY.md §8(d) concrete inputs).

Positions: a random walk per pedestrian starting at U(0,1)^2 (ETH pixel_pos
range) with N(0, 0.02^2) steps.  Frame f observes walk rows f .. f+T-1
(stride 1 sliding window, so the forward is recomputed every frame) and its
targets are the walk's next L rows f+T .. f+T+L-1.  vislet ~ N(0,1)
(UCY vislets are zero-mean standardised), G ~ N(0,1) (ctxt.png is absent from
the reference, Appendix B Q7), n_active ~ U{2..Nmax}.

Generated on the host with NumPy (seeded) so tests can hand the same arrays
to the oracle; ``to_device`` moves them into HBM before any timed region.
"""
from __future__ import annotations

from dataclasses import dataclass, fields

import numpy as np
import torch

from .frame_step import HIDDEN_LEN, OBS_LEN, PRED_LEN

# (name, S, Nmax, H, gpus) — BASELINE.json configs 2..5 (cfg 1 is real data)
CONFIGS = {
    "eth_hotel_synth": dict(S=256, Nmax=32, H=128),
    "eth_ucy_loo_kfold4": dict(S=1024, Nmax=64, H=128),   # 8 GPUs -> 128 per rank
    "relational_attn_h256": dict(S=256, Nmax=64, H=256),
    "dense_crowd": dict(S=1024, Nmax=256, H=256),          # 8 GPUs -> 128 per rank
}
FRAMES_PER_SCENE = OBS_LEN + PRED_LEN    # 20


@dataclass
class SceneBatch:
    pos: np.ndarray        # [S, W, Nmax, 2] f32
    vislet: np.ndarray     # [S, 2, Nmax]
    G: np.ndarray          # [S, D, T]
    targets: np.ndarray    # [S, F, Nmax, L, 2]
    n_active: np.ndarray   # [S] int32
    h0: np.ndarray         # [S, D, H]
    stride: int = 1
    n_frames: np.ndarray | None = None   # [S] int32 (real data: len(batch)); None: all F
    ped_mask: np.ndarray | None = None   # [S, Nmax] uint8 (real data); None: all active

    @property
    def frames(self) -> int:
        """Frames one step processes (the metric's unit)."""
        return int(self.n_frames.sum()) if self.n_frames is not None else self.S * self.F

    @property
    def S(self):
        return self.pos.shape[0]

    @property
    def F(self):
        return self.targets.shape[1]

    def to_device(self, device):
        out = {}
        for f in fields(self):
            v = getattr(self, f.name)
            out[f.name] = torch.from_numpy(np.ascontiguousarray(v)).to(device) \
                if isinstance(v, np.ndarray) else v
        return out


def make_batch(S, Nmax, H, *, F=FRAMES_PER_SCENE, seed=1, n_active=None, step_std=0.02,
               h0_scale=0.0) -> SceneBatch:
    rng = np.random.default_rng(seed)
    T, L, D = OBS_LEN, PRED_LEN, HIDDEN_LEN
    rows = (F - 1) + T + L
    start = rng.uniform(0.0, 1.0, size=(S, 1, Nmax, 2))
    steps = rng.normal(0.0, step_std, size=(S, rows - 1, Nmax, 2))
    walk = np.concatenate([start, start + np.cumsum(steps, axis=1)], axis=1).astype(np.float32)
    W = (F - 1) + T
    pos = np.ascontiguousarray(walk[:, :W])
    idx = np.arange(F)[:, None] + T + np.arange(L)[None, :]          # [F, L]
    targets = np.ascontiguousarray(np.transpose(walk[:, idx], (0, 1, 3, 2, 4)))  # [S,F,N,L,2]
    if n_active is None:
        n_active = rng.integers(2, Nmax + 1, size=S) if Nmax >= 2 else np.ones(S)
    n_active = np.asarray(n_active, dtype=np.int32)
    vislet = rng.standard_normal((S, 2, Nmax)).astype(np.float32)
    G = rng.standard_normal((S, D, T)).astype(np.float32)
    h0 = (h0_scale * rng.standard_normal((S, D, H))).astype(np.float32)
    return SceneBatch(pos=pos, vislet=vislet, G=G, targets=targets.astype(np.float32),
                      n_active=n_active, h0=h0, stride=1)
