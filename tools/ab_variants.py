"""Diagnostic A/B timing of g2k_step_fused_f32 build/env variants.

  python tools/ab_variants.py [--config NAME] [--rounds R] NAME=FLAGS[@ENV] ...

FLAGS are extra hipcc flags separated by ',' (e.g. -DG2K_POLL_SLEEP=0), ENV
are KEY:VALUE pairs separated by ',' applied while that variant runs (e.g.
G2K_SCENE_NP:12).  Each variant library is built into /tmp (never the shipped
one); variants are timed interleaved, R rounds of 50 steps, medians printed.
Also checks each variant's outputs against the first variant's.
"""
import argparse
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodaltraj_2_amd import _lib, build, frame_step as fs  # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="eth_hotel_synth")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("variants", nargs="+")
    args = ap.parse_args()
    vs = []
    for spec in args.variants:
        name, _, rest = spec.partition("=")
        flags, _, env = rest.partition("@")
        flags = [f for f in flags.split(",") if f]
        env = dict(kv.split(":", 1) for kv in env.split(",") if kv)
        out = f"/tmp/libg2k_ab_{name}.so"
        subprocess.run([build.HIPCC, *build.FLAGS, *flags, "-o", out, *build.SRC], check=True)
        vs.append((name, _lib.load(out), env))
    c = CONFIGS[args.config]
    S = c["S"] if c["S"] <= 256 else c["S"] // 8
    b = make_batch(S, c["Nmax"], c["H"])
    dev = torch.device("cuda")
    p = fs.init_params(c["Nmax"], device=dev)
    t = b.to_device(dev)
    res = {v[0]: [] for v in vs}
    outs = {}
    for rnd in range(args.rounds):
        for name, lib, env in vs:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            _lib._lib = lib
            try:
                plan = fs.StepPlan(p, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
                o = plan.out
                for _ in range(3):
                    plan.run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                for _ in range(50):
                    plan.run()
                e1.record()
                torch.cuda.synchronize()
                res[name].append(e0.elapsed_time(e1) / 50 * 1e3)
                if rnd == 0:
                    outs[name] = (o.pred.cpu(), o.h.cpu(), o.metrics.cpu())
            finally:
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
    ref = outs[vs[0][0]]
    for name, _, _ in vs:
        o = outs[name]
        d = [float((x - y).abs().max()) for x, y in zip(o, ref)]
        print(f"{name:16s} median {np.median(res[name]):8.2f} us  min {min(res[name]):8.2f}  "
              f"max|d| vs {vs[0][0]}: pred {d[0]:.2e} h {d[1]:.2e} metrics {d[2]:.2e}")


if __name__ == "__main__":
    main()
