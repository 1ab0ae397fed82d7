"""Diagnostic: max relative-to-max(1,|ref|) error of every output of the fused
step vs the float64 oracle, over several geometries."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_step_gpu import run_both
from tests.conftest import close
dev = torch.device("cuda")
for (S, N, H) in [(4, 32, 128), (3, 64, 256), (2, 256, 128), (2, 256, 256)]:
    b, out, res = run_both(S, N, H, device=dev, h0_scale=1.0)
    e = {k: 0.0 for k in ("pred", "attn", "cost", "h", "metrics")}
    for s in range(S):
        n = int(b.n_active[s]); pr, h, m, ex = res[s]
        e["pred"] = max(e["pred"], close(out.pred[s, :, :, :n].cpu().numpy().reshape(-1, 2, 12, n), pr))
        e["attn"] = max(e["attn"], close(out.attn[s].cpu().numpy(), np.stack(ex["A"])))
        e["cost"] = max(e["cost"], close(out.cost[s].cpu().numpy(), np.stack(ex["cost"])))
        e["h"] = max(e["h"], close(out.h[s].cpu().numpy(), h))
        e["metrics"] = max(e["metrics"], close(out.metrics[s, :6].cpu().numpy(), m[:6]))
    print(S, N, H, {k: f"{v:.2e}" for k, v in e.items()}, "n_active", b.n_active.tolist())
