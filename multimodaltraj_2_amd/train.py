"""train.py entry point (train.py:17-695: the training leg over the k-fold
datasets, then the leave-one-out validation leg), per-frame body on the GPU
through g2k_step_fused_f32.

  python -m multimodaltraj_2_amd.train --data_root /path/to/data [flags of argParser]

Training leg (train.py:27-365): for every dataset except --leaveDataset and
every epoch it walks the DataLoader batches, builds the online graph, runs the
batch's frame loop as one fused HIP step (hidden state carried from batch to
batch when --chain_hidden, like train.py's ``hidden_state``) with the training
log's pairing (prediction row i against the (i-1)-th target key,
train.py:257-276), and writes the reference's raw-vector logs
<log_dir>/g2k_MPC_error_log_kfold_<d>.csv (every logged difference row,
raveled) and g2k_MPC_fde_log_kfold_<d>.csv (one final-step difference per
row) after every epoch (train.py:346-351), the counts file
g2k_lstm_counts_<d>.txt (:361-364) and, as the build's own summary,
g2k_MPC_batch_metrics_kfold_<d>.csv (epoch, batch, ADE, FDE, num_peds of the
kernel's a9 error terms).  With --save_dir the weights are written as TF
tensor bundles under the reference's variable and file names, with its
global-step cadence and ``checkpoint`` state file (train.py:330-343;
multimodaltraj_2_amd/checkpoint.py).

Validation leg (train.py:371-695): the left-out dataset's batches from the
valid pointers (:408-411), validation pairing (row i against key i), hidden
state chained across batches, cross-validation ADE / FDE per batch (:668-674,
FDE divided by num_nodes when the left-out dataset is 5) and their means, and
the g2k_MPC_model_kfold_val_<l>.ckpt checkpoint (:688-691).

The model weights are one seeded N(0, 1) draw (quirk Q15: the reference
re-draws them every batch).
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
from .scenes import build_scene, pack, train_log_vectors


def _g(seed, D, device):
    """The context input _2dconv_in [D, T]: ctxt.png is absent (quirk Q7),
    a seeded N(0, 1) stand-in."""
    return torch.from_numpy(np.random.default_rng(seed + 1).standard_normal(
        (1, D, fs.OBS_LEN)).astype(np.float32)).to(device)


def _step(args, sc, params_cache, h, device):
    pk = pack([sc], args.rnn_size)
    key = pk["Nmax"]
    if key not in params_cache:
        params_cache[key] = fs.init_params(key, seed=args.seed, device=device)
    t = {k: torch.from_numpy(v).to(device) for k, v in pk.items() if isinstance(v, np.ndarray)}
    out = fs.step_fused(params_cache[key], t["pos"], t["vislet"], _g(args.seed, fs.HIDDEN_LEN, device),
                        t["targets"], t["n_active"], h, n_frames=t["n_frames"],
                        ped_mask=t["ped_mask"], stride=0, lam=args.lambda_param)
    return out, params_cache[key]


class TrainLog:
    """The training leg's raw-vector logs (train.py:27-30, 254-276, 346-351):
    euc_loss / fde lists shared by every dataset of the fold (as the
    reference's, initialised once per left-out dataset) and per-dataset step
    counts."""

    def __init__(self):
        self.euc, self.fde = [], []
        self.num_targets = self.num_end_targets = 0

    def add(self, pred, n_frames, n, target_traj):
        """pred [F, 2L, Nmax] (device) of one batch; one frame's rows per frame
        of the batch's loop (train.py:197)."""
        p = pred[:n_frames, :, :n].detach().cpu().numpy().reshape(n_frames, 2, fs.PRED_LEN, n)
        for f in range(n_frames):
            self.num_targets += n
            self.num_end_targets += max(0, min(n - 1, len(target_traj)))
            e, d = train_log_vectors(p[f], target_traj, fs.PRED_LEN)
            self.euc += e
            self.fde += d

    def write(self, log_dir, d):
        if self.fde:
            np.savetxt(os.path.join(log_dir, f"g2k_MPC_fde_log_kfold_{d}.csv"), np.stack(self.fde),
                       delimiter=",")
        if self.euc:
            np.savetxt(os.path.join(log_dir, f"g2k_MPC_error_log_kfold_{d}.csv"),
                       np.concatenate([np.ravel(e) for e in self.euc]), delimiter=",")


def run_dataset(args, d, params_cache, device, log, tlog=None, loader=None, graph=None):
    """Training leg for dataset d.  Returns (rows, last frame key, graph)."""
    loader = loader or DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=d, sel=0,
                                  data_root=args.data_root)
    graph = graph or nxg.online_graph(args)
    tlog = tlog if tlog is not None else TrainLog()
    h = torch.zeros((1, 16, args.rnn_size), device=device)
    rows = []
    frame = 1                                                # train.py:34
    for e in range(args.num_epochs):
        loader.reset_data_pointer()
        t0 = time.time()
        for b in range(loader.num_batches):
            batch, tgt, _ = loader.next_step()
            if len(batch) == 0:
                break
            g = graph.ConstructGraph(current_batch=batch, framenum=int(frame), future_traj=tgt)
            sc = build_scene(batch, tgt, g, loader, frame, mode=args.slice, pairing="train_log")
            for k in batch:                                  # train.py:197 leaves frame = last key
                frame = k
            n = sc.window.shape[1]
            if n < 2:                                        # train.py:86-90: batch skipped
                continue
            out, params = _step(args, sc, params_cache, h, device)
            if args.chain_hidden:
                h = out.h
            tlog.add(out.pred[0], sc.n_frames, n, tgt)
            ade, fde = fs.batch_errors(out.metrics, leave_dataset=args.leaveDataset, num_nodes=[n])
            rows.append((e, b, float(ade[0]), float(fde[0]), n))
            if args.save_dir and checkpoint.save_due(e, b, loader.num_batches, args.save_every):
                checkpoint.save_params(checkpoint.checkpoint_prefix(args.save_dir, d, e, b, loader.num_batches),
                                       params)               # train.py:330-341
        if args.log_dir:
            tlog.write(args.log_dir, d)                      # train.py:346-351, every epoch
        log(f"dataset {d} epoch {e}: {len(rows)} batches, {time.time() - t0:.2f}s")
    return rows, frame, graph


def validate(args, frame, graph, params_cache, device, log=print, loader=None, start_pointer=0):
    """The validation leg on dataset l = --leaveDataset (train.py:371-695).
    Returns (cv_ade_err, cv_fde_err) per validation batch.  ``start_pointer``:
    the reference resets the frame pointer to 0 (reset_data_pointer(valid=True),
    :377); on the ETH/UCY files, whose frame keys are 1 + 8k (zara02: 7 + 8k),
    no key is ever found from there and the leg sees no batch (its means are
    nan).  ``start_pointer=None`` starts at the file's first frame instead
    (build option, --valid_from_seed)."""
    l = args.leaveDataset
    loader = loader or DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=l, sel=0,
                                  data_root=args.data_root)
    loader.reset_data_pointer(valid=True, frame_pointer=loader.seed if start_pointer is None else start_pointer)
    loader.valid_frame_pointer = int((loader.len - int(loader.max * .7)) / loader.val_max)   # :408-409
    loader.valid_num_batches = int(loader.val_max / loader.batch_size)                    # :411
    graph = graph or nxg.online_graph(args)
    h = torch.zeros((1, 16, args.rnn_size), device=device)
    cv_ade_err, cv_fde_err = [], []
    vb = 0
    for vb in range(loader.valid_num_batches):
        batch, tgt, fp = loader.next_step()
        if len(batch) == 0:
            break
        g = graph.ConstructGraph(current_batch=batch, framenum=fp, future_traj=tgt)
        sc = build_scene(batch, tgt, g, loader, frame, mode=args.slice, pairing="row",
                         vislet_offset=loader.valid_frame_pointer)
        n = sc.window.shape[1]
        if n < 1:
            break                                            # :437-442
        out, params = _step(args, sc, params_cache, h, device)
        h = out.h                                            # hidden_state carried (:558-575)
        ade, fde = fs.batch_errors(out.metrics, leave_dataset=l, num_nodes=[n])
        if np.isfinite(ade[0]):
            cv_ade_err.append(float(ade[0]))
            cv_fde_err.append(float(fde[0]))
        for k in batch:
            frame = k
        loader.frame_pointer = frame                         # :682
    if cv_ade_err:
        log(f"Cross-Validation total mean error (ADE) for dataset {l} = {np.mean(cv_ade_err)}")
        log(f"Cross-Validation total final error (FDE) for dataset {l} = {np.mean(cv_fde_err)}")
    if args.save_dir and params_cache:
        e = max(args.num_epochs - 1, 0)
        prefix = os.path.join(args.save_dir, f"g2k_MPC_model_kfold_val_{l}.ckpt-"
                                             f"{e * loader.valid_num_batches + vb}")
        checkpoint.save_params(prefix, next(iter(params_cache.values())))   # :688-691
    return cv_ade_err, cv_fde_err


def train(args):
    device = torch.device(args.device)
    os.makedirs(args.log_dir, exist_ok=True)
    datasets = {2, 3, 4, 5} - {args.leaveDataset}
    cache = {}
    tlog = TrainLog()
    frame, graph = 1, None
    for d in sorted(datasets):
        tlog.num_targets = tlog.num_end_targets = 0
        try:
            rows, frame, graph = run_dataset(args, d, cache, device, print, tlog)
        except FileNotFoundError as exc:                   # town_center.csv (5) is absent
            print(f"dataset {d}: {exc}")
            continue
        path = os.path.join(args.log_dir, f"g2k_MPC_batch_metrics_kfold_{d}.csv")
        np.savetxt(path, np.array(rows, dtype=np.float64).reshape(-1, 5), delimiter=",")
        with open(os.path.join(args.log_dir, f"g2k_lstm_counts_{d}.txt"), "w") as f:
            f.write(f"Dataset {d}= ADE steps {tlog.num_targets}\nFDE steps = {tlog.num_end_targets}")
        ok = [r for r in rows if np.isfinite(r[2])]
        if ok:
            print(f"dataset {d}: mean ADE {np.mean([r[2] for r in ok]):.4f} "
                  f"mean FDE {np.mean([r[3] for r in ok]):.4f} ({len(ok)} batches)")
    try:
        validate(args, frame, graph, cache, device,
                 start_pointer=None if getattr(args, "valid_from_seed", 0) else 0)
    except FileNotFoundError as exc:
        print(f"validation dataset {args.leaveDataset}: {exc}")


def main(argv=None):
    args = ArgsParser().parser.parse_args(argv)
    train(args)


if __name__ == '__main__':
    main()
