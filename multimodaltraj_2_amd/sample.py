"""sample.py entry point (sample.py:85-355): one forward per batch through the
HIP step (a fresh online graph per batch, framenum 0, time slice of the
node positions, sample.py:150-164) and get_mean_error (sample.py:21-82) on the
GPU (g2k_ade_fde_f32 variant 1).

  python -m multimodaltraj_2_amd.sample --data_root /path/to/data --test_dataset 2
"""
from __future__ import annotations

import argparse

import numpy as np
import torch

from . import frame_step as fs
from . import networkx_graph as nxg
from .argParser import ArgsParser
from .load_traj import DataLoader
from .scenes import build_scene, pack


def main(argv=None):
    base = ArgsParser().parser
    p = argparse.ArgumentParser(parents=[base], add_help=False, conflict_handler="resolve")
    p.add_argument('--obs_length', type=int, default=8)
    p.add_argument('--pred_length', type=int, default=12)
    p.add_argument('--test_dataset', type=int, default=2)
    p.add_argument('--epoch', type=int, default=2)
    args = p.parse_args(argv)
    device = torch.device(args.device)
    loader = DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=args.test_dataset, sel=0,
                        data_root=args.data_root)
    loader.reset_data_pointer()
    H = args.rnn_size
    total, final = [], []
    for b in range(loader.num_batches):
        batch, tgt, _ = loader.next_step()
        if len(batch) == 0:
            break
        g = nxg.online_graph(args).ConstructGraph(current_batch=batch, framenum=0, future_traj=tgt)
        sc = build_scene(batch, tgt, g, loader, 0, mode="sample")
        node_t = g.get_node_attr("targets")
        try:
            y = np.stack([np.asarray(v[0], np.float64) for v in node_t.values()])
        except ValueError:
            continue                                       # ragged targets: np.stack fails too
        if y.ndim != 3 or y.shape[1] < 12:
            continue
        sc.targets = y[:, :12]
        sc.mask[:] = True
        sc.n_frames = 1
        pk = pack([sc], H)
        params = fs.init_params(pk["Nmax"], seed=args.seed, device=device)
        t = {k: torch.from_numpy(v).to(device) for k, v in pk.items() if isinstance(v, np.ndarray)}
        G = torch.from_numpy(np.random.default_rng(args.seed + 1).standard_normal(
            (1, 16, 8)).astype(np.float32)).to(device)
        h = torch.zeros((1, 16, H), device=device)
        out = fs.step_fused(params, t["pos"], t["vislet"], G, t["targets"], t["n_active"], h,
                            n_frames=t["n_frames"], stride=0, lam=args.lambda_param)
        err = fs.ade_fde(out.pred[:, 0].contiguous(), t["targets"][:, 0].contiguous(),
                         t["n_active"], variant=1, obs_length=args.obs_length)
        e = err[0].cpu().numpy()
        total.append(float(e[0]))
        final.append(float(e[1]))
        print(f"batch {b}: ADE {e[0]:.4f} FDE {e[1]:.4f} peds {sc.window.shape[1]}")
    if total:
        print("Total mean error of the model is ", np.mean(total))
        print("Total final error of the model is ", np.mean(final))


if __name__ == '__main__':
    main()
