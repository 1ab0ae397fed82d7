"""sample.py entry point (sample.py:85-355) at the reference's geometry:
D = num_freq_blocks (10), one g2k_lstm_mcr forward per batch on the GPU
(g2k_mcr_forward_f32 at D = 10, the GridLSTM encoder through g2k_gridlstm_f32)
and get_mean_error (sample.py:21-82) through g2k_ade_fde_f32 variant 1.

  python -m multimodaltraj_2_amd.sample --data_root /path/to/data --test_dataset 2 \\
      [--save_dir save]          # restore krnl_weights from the latest checkpoint

Per batch (sample.py:137-330):
  * a fresh online graph at framenum 0, the time slice of the node positions
    (sample.py:150-164) -> batch_v = ||pos|| [obs_len, n];
  * weight_i [n, D], weight_ii [D, obs_len] ~ N(0, 1) (:186-195), inputs =
    weight_ii @ (batch_v @ weight_i) [D, D], vislet_emb = vislet @ weight_i
    [2, D], vislet_rel = vislet_past * vislet_emb (:141-144, :197-201);
  * the GridLSTM encoder over inputs with a zero state (:262-269, helper.py:
    10-75; 2 blocks of 4 of the 10 columns, tf.contrib's slicing) -> ng_output
    [D, 8];
  * g2k_lstm_mcr.forward with outputs = [inputs; vislet_emb], ngh = lambda *
    ng_output (scaled by lambda again inside the model, :102, as the reference
    feeds it), rel_features = vislet_rel (:297-312);
  * get_mean_error(complete_traj, targets) (:327-332).
Weights: krnl_weights / krnl_embed restored from the checkpoint the
``checkpoint`` state file in --save_dir names (sample.py:213-225;
checkpoint.load_params), pedestrian columns the checkpoint lacks (its weight_o
is sized by the saving batch) drawn N(0, 1); without --save_dir all are drawn
N(0, 1).  Build decision: the reference re-initialises the restored variables
right after restoring them (:294-296, quirk) — the restore is kept effective
here.  The static-context branch (:271-290) feeds nothing the prediction reads
and is not run.  Small glue products (weight_ii @ batch_v @ weight_i, the
vislet embedding) are torch matmuls on the GPU.
"""
from __future__ import annotations

import argparse
import os

import numpy as np
import torch

from . import checkpoint
from . import frame_step as fs
from . import helper
from . import networkx_graph as nxg
from .argParser import ArgsParser
from .load_traj import DataLoader
from .models.g2k_lstm_mcr import g2k_lstm_mcr
from .scenes import build_scene


def restore_weights(save_dir, device):
    """The krnl_* variables of the latest checkpoint in save_dir (G2KParams,
    float32 on device) or None (no state file)."""
    prefix = checkpoint.read_state(save_dir) if save_dir else None
    if prefix is None:
        return None
    return checkpoint.load_params(prefix, device=device)


def model_weights(restored, n, D, T, seed, device, log=print):
    """g2k_lstm_mcr weights for a batch of n pedestrians: the restored ones,
    weight_o's missing columns (and everything without a checkpoint) N(0, 1).
    A checkpoint of another hidden_len (train.py writes D = 16, sample.py runs
    D = num_freq_blocks = 10) cannot be used: N(0, 1) weights, with a warning."""
    rng = np.random.default_rng(seed)
    draw = lambda shape: torch.from_numpy(rng.standard_normal(shape).astype(np.float32)).to(device)
    w = dict(weight_v=draw((T, D + 2)), bias_v=draw((D,)), weight_o=draw((T, n)),
             weight_c=draw((2 * fs.PRED_LEN, T)), weight_r=draw((T, 2)))
    if restored is not None and tuple(restored.Wv.shape) != (T, D + 2):
        log(f"checkpoint weight_v {tuple(restored.Wv.shape)} is not [{T}, {D + 2}] (D = "
            f"num_freq_blocks = {D}): its weights are not used, N(0, 1) instead")
        restored = None
    if restored is not None:
        k = min(n, int(restored.Wo.shape[1]))
        wo = w["weight_o"].clone()
        wo[:, :k] = restored.Wo[:, :k]
        w = dict(weight_v=restored.Wv, bias_v=restored.bv, weight_o=wo, weight_c=restored.Wc,
                 weight_r=restored.Wr)
    return w


class StageTimer:
    """Per-stage wall times of sample.py:256-325 by HIP events on the current
    stream (the reference's time.time() prints become hipEvent
    timers): ``mark(name)`` closes the stage running since the previous mark;
    ``seconds()`` synchronises once and returns {stage: seconds}."""

    def __init__(self, device):
        self.device = device
        self.events = []
        self.t0 = self._event()

    def _event(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def mark(self, name):
        self.events.append((name, self._event()))

    def seconds(self):
        self.events[-1][1].synchronize()
        out, prev = {}, self.t0
        for name, e in self.events:
            out[name] = prev.elapsed_time(e) / 1e3
            prev = e
        out["total"] = self.t0.elapsed_time(self.events[-1][1]) / 1e3
        return out


def sample_batch(args, sc, vislet_past, restored, device, seed, timer=None):
    """One batch of sample.py (see the module docstring).  Returns
    (ade, fde, vislet_emb, pred [2, 12, n]) — errors from g2k_ade_fde_f32.
    ``timer`` (StageTimer): the stages of sample.py:256-325 are marked on it."""
    D, T = args.num_freq_blocks, args.obs_len
    n = sc.window.shape[1]
    rng = np.random.default_rng(seed)
    tt = lambda a: torch.as_tensor(np.asarray(a, np.float32), device=device)
    mark = timer.mark if timer is not None else (lambda name: None)
    batch_v = np.linalg.norm(sc.window, axis=2)                     # [obs_len, n]
    weight_i = tt(rng.standard_normal((n, D)))
    weight_ii = tt(rng.standard_normal((D, batch_v.shape[0])))
    inputs = weight_ii @ (tt(batch_v) @ weight_i)                   # [D, D]
    vislet_emb = tt(sc.vislet[:, :n]) @ weight_i                    # [2, D]
    vislet_rel = vislet_past * vislet_emb
    enc = helper.neighborhood_vis_loc_encoder(hidden_size=args.rnn_size, hidden_len=D,
                                              num_layers=args.num_layers, grid_size=args.grid_size,
                                              embedding_size=args.embedding_size, device=device,
                                              seed=seed)
    model = g2k_lstm_mcr(in_features=(D, D), hidden_size=args.rnn_size, obs_len=T, num_nodes=n,
                         lambda_reg=args.lambda_param, device=device,
                         weights=model_weights(restored, n, D, T, seed + 1, device))
    mark("setup")
    ng_output, _ = enc.forward(inputs.contiguous(), torch.zeros((D, args.rnn_size), device=device))
    mark("social")                                                  # sample.py:258-268
    mark("static")                                                  # :273-282 (not run, see main)
    mark("combined")                                                # :284-291 (not run)
    pred = model.forward(dict(outputs=torch.cat([inputs, vislet_emb], 0), ngh=args.lambda_param * ng_output,
                              rel_features=vislet_rel, out_size=n))
    mark("predictive")                                              # :300-310
    mark("relational")                                              # :313-322 (no op in the reference)
    nmax = max(n, 1)
    pr = torch.zeros((1, 2 * fs.PRED_LEN, nmax), device=device)
    pr[0, :, :n] = model.temp_path
    tg = torch.zeros((1, nmax, fs.PRED_LEN, 2), device=device)
    tg[0, :n] = tt(sc.targets)
    err = fs.ade_fde(pr, tg, torch.tensor([n], dtype=torch.int32, device=device), variant=1,
                     obs_length=args.obs_length)
    mark("errors")                                                  # :326-330
    e = err[0].cpu().numpy()
    return float(e[0]), float(e[1]), vislet_emb, pred


def batches(args, loader):
    """sample.py:137-164 / 318-320: (batch index, scene, the batch's frame
    dict x_batch) per batch with targets."""
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
        if y.ndim != 3 or y.shape[1] < fs.PRED_LEN or sc.window.shape[1] < 1:
            continue
        sc.targets = y[:sc.window.shape[1], :fs.PRED_LEN]
        yield b, sc, batch


STAGE_LINES = (   # sample.py:268, 282, 291, 310, 322, 325 (wording kept)
    ("social", "wall-clock time taken by social mask grid = {0} seconds"),
    ("static", "wall-clock time taken by static mask grid = {0} seconds"),
    ("combined", "wall-clock time taken by combined mask grid = {0} seconds"),
    ("predictive", "wall-clock time taken by predictive kernel = {0} seconds"),
    ("relational", "Relational inference calculation took= {0} seconds"),
)


def run(args, loader, device, log=print):
    """sample.py:137-340: every batch, its stage timings (hipEvents), its
    errors; returns (total, final, results) with results =
    [(x_batch, complete_traj [n, 12, 2], obs_length)] as sample.py:340 builds it."""
    restored = restore_weights(args.save_dir, device)
    vislet_past = 1.0
    total, final, results = [], [], []
    for b, sc, x_batch in batches(args, loader):
        log("********************** SAMPLING A NEW TRAJECTORY", b,
            "******************************")
        timer = StageTimer(device)
        ade, fde, vislet_past, pred = sample_batch(args, sc, vislet_past, restored, device,
                                                   args.seed, timer)
        sec = timer.seconds()
        for key, line in STAGE_LINES:
            log(line.format(sec[key]))
        # start -> end of sample.py:256-325 (the model's stages, not the errors)
        log("Multi-Cued model (MCR) sampling time = {0} seconds".format(
            sum(sec[k] for k, _ in STAGE_LINES)))
        total.append(ade)
        final.append(fde)
        log(f"batch {b}: ADE {ade:.4f} FDE {fde:.4f} peds {sc.window.shape[1]}")
        log("Processed trajectory number : ", b, "out of ", loader.num_batches, " trajectories")
        complete_traj = np.transpose(pred.detach().cpu().numpy(), (2, 1, 0))   # sample.py:326
        results.append((x_batch, complete_traj, args.obs_length))              # :340
    return total, final, results


def save_results(results, save_dir, log=print):
    """sample.py:346-348: pickle.dump(results) to <save dir>/social_results.pkl
    (the reference's hard-coded save directory is --save_dir here, Q8;
    the current directory without one).  Returns the path."""
    import pickle
    log("Saving results")
    os.makedirs(save_dir or ".", exist_ok=True)
    path = os.path.join(save_dir or ".", "social_results.pkl")
    with open(path, "wb") as f:
        pickle.dump(results, f)
    return path


def parse_args(argv=None):
    """argParser.py's flags plus sample.py's own (sample.py:89-106), same
    names and defaults."""
    base = ArgsParser().parser
    p = argparse.ArgumentParser(parents=[base], add_help=False, conflict_handler="resolve")
    p.add_argument('--obs_length', type=int, default=8)
    p.add_argument('--pred_length', type=int, default=12)
    p.add_argument('--test_dataset', type=int, default=5)   # sample.py:98 (5: town_center.csv)
    p.add_argument('--epoch', type=int, default=2)
    return p.parse_args(argv)


def main(argv=None):
    args = parse_args(argv)
    device = torch.device(args.device)
    # dataset 5 is town_center.csv (load_traj.py:30), which the reference's data/
    # does not ship: the loader raises FileNotFoundError there, as the
    # reference's np.genfromtxt does
    loader = DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=args.test_dataset, sel=0,
                        data_root=args.data_root)
    loader.reset_data_pointer()
    if args.save_dir and not os.path.exists(os.path.join(args.save_dir, "checkpoint")):
        print(f"no checkpoint state file in {args.save_dir}: weights drawn N(0, 1)")
    print("static / combined mask grid stages: not run (their outputs feed nothing the "
          "prediction reads, and the reference's stat_mask [dim, num_freq_blocks] + [8, 1] "
          "does not broadcast: sample.py:181-182); timed as empty stages")
    total, final, results = run(args, loader, device)
    if total:
        print("Total mean error of the model is ", np.mean(total))
        print("Total final error of the model is ", np.mean(final))
    save_results(results, args.save_dir)
    return total, final, results


if __name__ == '__main__':
    main()
