"""train.py entry point (train.py:17-365 training loop, per-frame body on the
GPU through g2k_step_fused_f32).

  python -m multimodaltraj_2_amd.train --data_root /path/to/data [flags of argParser]

For every dataset except --leaveDataset (train.py:38-39) and every epoch it
walks the DataLoader batches, builds the online graph, runs the batch's frame
loop as one fused HIP step (hidden state carried from batch to batch when
--chain_hidden, like train.py's ``hidden_state``), and writes per-batch
ADE / FDE rows ``epoch,batch,ADE,FDE,num_peds`` to
<log_dir>/g2k_MPC_error_log_kfold_<d>.csv.  The model weights are one seeded
N(0, 1) draw (quirk Q15: the reference re-draws them every batch).  With
--save_dir they are written as TF tensor bundles under the reference's
variable names and file names, with its global-step cadence and ``checkpoint``
state file (train.py:330-343; multimodaltraj_2_amd/checkpoint.py).
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import checkpoint
from . import frame_step as fs
from . import networkx_graph as nxg
from .argParser import ArgsParser
from .load_traj import DataLoader
from .scenes import build_scene, pack


def run_dataset(args, d, params_cache, device, log):
    loader = DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=d, sel=0, data_root=args.data_root)
    graph = nxg.online_graph(args)
    H = args.rnn_size
    h = torch.zeros((1, 16, H), device=device)
    rows = []
    for e in range(args.num_epochs):
        loader.reset_data_pointer()
        frame = 1                                            # train.py:34
        t0 = time.time()
        for b in range(loader.num_batches):
            batch, tgt, _ = loader.next_step()
            if len(batch) == 0:
                break
            g = graph.ConstructGraph(current_batch=batch, framenum=int(frame), future_traj=tgt)
            sc = build_scene(batch, tgt, g, loader, frame, mode=args.slice)
            for k in batch:                                  # train.py:197 leaves frame = last key
                frame = k
            n = sc.window.shape[1]
            if n < 2:                                        # train.py:86-90: batch skipped
                continue
            pk = pack([sc], H)
            key = pk["Nmax"]
            if key not in params_cache:
                params_cache[key] = fs.init_params(key, seed=args.seed, device=device)
            t = {k: torch.from_numpy(v).to(device) for k, v in pk.items() if isinstance(v, np.ndarray)}
            G = torch.from_numpy(np.random.default_rng(args.seed + 1).standard_normal(
                (1, 16, 8)).astype(np.float32)).to(device)   # ctxt.png absent (Q7)
            out = fs.step_fused(params_cache[key], t["pos"], t["vislet"], G, t["targets"],
                                t["n_active"], h, n_frames=t["n_frames"], ped_mask=t["ped_mask"],
                                stride=0, lam=args.lambda_param)
            if args.chain_hidden:
                h = out.h
            ade, fde = fs.batch_errors(out.metrics, leave_dataset=args.leaveDataset, num_nodes=[n])
            rows.append((e, b, float(ade[0]), float(fde[0]), n))
            if args.save_dir and checkpoint.save_due(e, b, loader.num_batches, args.save_every):
                checkpoint.save_params(checkpoint.checkpoint_prefix(args.save_dir, d, e, b, loader.num_batches),
                                       params_cache[key])     # train.py:330-341
        log(f"dataset {d} epoch {e}: {len(rows)} batches, {time.time() - t0:.2f}s")
    return rows


def train(args):
    device = torch.device(args.device)
    os.makedirs(args.log_dir, exist_ok=True)
    datasets = {2, 3, 4, 5} - {args.leaveDataset}
    cache = {}
    for d in sorted(datasets):
        try:
            rows = run_dataset(args, d, cache, device, print)
        except FileNotFoundError as exc:                   # town_center.csv (5) is absent
            print(f"dataset {d}: {exc}")
            continue
        path = os.path.join(args.log_dir, f"g2k_MPC_error_log_kfold_{d}.csv")
        np.savetxt(path, np.array(rows, dtype=np.float64).reshape(-1, 5), delimiter=",")
        ok = [r for r in rows if np.isfinite(r[2])]
        if ok:
            print(f"dataset {d}: mean ADE {np.mean([r[2] for r in ok]):.4f} "
                  f"mean FDE {np.mean([r[3] for r in ok]):.4f} ({len(ok)} batches)")


def main(argv=None):
    args = ArgsParser().parser.parse_args(argv)
    train(args)


if __name__ == '__main__':
    main()
