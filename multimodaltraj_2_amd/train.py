"""train.py entry point (train.py:17-695), per-frame body on the GPU.

  python -m multimodaltraj_2_amd.train --data_root DIR [flags of argParser]
  torchrun --nproc-per-node K -m multimodaltraj_2_amd.train --mode train --world_size K ...

--mode reference (default): the reference's two legs.
  Training leg (train.py:27-365).  The data walk is the reference's
  (walks.train_walk: graph per dataset, the node slice of train.py:78, the
  batch_v checks, the second ConstructGraph of every batch, epochs).  As in the
  reference, the epoch counter ``e``, ``frame`` and the step counters are set
  once per left-out dataset (train.py:29-36), so the epochs all run on the
  fold's first dataset and the later datasets only write their counts files.
  Every epoch's batches go to the GPU in ONE g2k_step_fused_f32 launch (stride
  0: the reference feeds each batch's window to every frame of its loop), and
  the hidden state is chained through all of them, batch after batch and epoch
  after epoch as train.py carries ``hidden_state``, by one
  g2k_frame_recurrence_f32 launch over the epoch's attention matrices in frame
  order (pred and the errors never read h, so nothing else is sequential).  The
  training log's pairing (prediction row i against the (i-1)-th target key,
  train.py:257-276) gives the raw-vector logs <log_dir>/g2k_MPC_error_log_kfold
  _<d>.csv and g2k_MPC_fde_log_kfold_<d>.csv after every epoch (:346-351), the
  counts file g2k_lstm_counts_<d>.txt (:361-364) and, as the build's summary,
  g2k_MPC_batch_metrics_kfold_<d>.csv.  With --save_dir: TF tensor bundles
  under the reference's names, file names and cadence (:330-343).
  Validation leg (train.py:371-695): a fresh graph and frame = 1 (:374, :392),
  the left-out dataset's walk (walks.valid_walk; the reference's pointer 0
  finds no key of the ETH/UCY files, --valid_from_seed starts at the first
  frame), all its batches in one launch, the hidden state chained from zeros,
  validation pairing (row i against key i), per-batch cross-validation ADE /
  FDE (:668-674, FDE / num_nodes when the left-out dataset is 5) and their
  means, and the g2k_MPC_model_kfold_val_<l>.ckpt checkpoint (:688-693).

--use_grid_lstm 1 (default 0 = the reference,
  whose encoder outputs are overridden by feeds): both legs run the vis/loc
  encoder's GridLSTMCell in every frame (train.py:201-207 with its output as
  st_embeddings), one sequential chain per leg (encoder_step.EncoderChain).

--mode train (the build's; the reference has no loss or optimizer): RMSProp
  (--learning_rate, --decay_rate, --grad_clip; argParser.py:38-47) on the L2
  loss of the predictions or (--loss nll) the bivariate-Gaussian NLL with a
  learned per-step head, over the fold's real scenes (realdata.plan_scenes:
  sample.py's scene per frame pointer, every distinct window of the training
  datasets), --train_batch scenes per global step, each rank taking its
  contiguous shard (dist.shard_scenes) and ONE all-reduce of the flat gradient
  per step (RCCL under torchrun with the nccl backend), then the same update on
  every rank.

The model weights are one seeded N(0, 1) draw (quirk Q15: the reference
re-draws them every batch), padded to Nmax (8 for the node slice).
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import checkpoint
from . import frame_step as fs
from . import walks
from .argParser import ArgsParser
from .load_traj import DataLoader
from .scenes import pack, scene_from_record, train_log_vectors

NODE_SLICE_NMAX = 8      # the node slice [frame:frame+obs_len] holds at most obs_len nodes


def context_G(seed, S=1, D=fs.HIDDEN_LEN):
    """_2dconv_in [S, D, T] (train.py:158): ctxt.png is absent (quirk Q7), a
    seeded N(0, 1) stand-in, the same for every batch of a run."""
    g = np.random.default_rng(seed + 1).standard_normal((1, D, fs.OBS_LEN)).astype(np.float32)
    return np.repeat(g, S, axis=0)


class TrainLog:
    """The training leg's raw-vector logs (train.py:30-32, 254-276, 346-351):
    euc_loss / fde lists initialised once per left-out dataset, one entry per
    logged pair and frame."""

    def __init__(self):
        self.euc, self.fde = [], []

    def add(self, pred_band, n_frames, target_traj):
        """pred_band [2, L, n] (host) of one batch: the batch's frame loop logs
        the same rows once per frame (its inputs do not change within a
        batch, train.py:197-276)."""
        e, d = train_log_vectors(pred_band, target_traj, fs.PRED_LEN)
        for _ in range(n_frames):
            self.euc += e
            self.fde += d

    def write(self, log_dir, d):
        if self.fde:
            np.savetxt(os.path.join(log_dir, f"g2k_MPC_fde_log_kfold_{d}.csv"), np.stack(self.fde),
                       delimiter=",")
        if self.euc:
            np.savetxt(os.path.join(log_dir, f"g2k_MPC_error_log_kfold_{d}.csv"),
                       np.concatenate([np.ravel(e) for e in self.euc]), delimiter=",")


def encoder_cell(args, device):
    """--use_grid_lstm: the vis/loc encoder's cell (helper.py:19-39 as
    train.py:119-125 builds it: num_units = --num_layers, feature_size =
    --grid_size, D / grid_size frequency blocks), seeded weights (the
    reference's initialisers are unseeded)."""
    from .helper import neighborhood_vis_loc_encoder
    return neighborhood_vis_loc_encoder(hidden_size=args.rnn_size, hidden_len=fs.HIDDEN_LEN,
                                        num_layers=args.num_layers, grid_size=args.grid_size,
                                        embedding_size=args.embedding_size, dropout=args.dropout,
                                        device=device, seed=args.seed).rnn


def launch_records(args, recs, loader, params, device, h, pairing, cell=None):
    """The batches of one epoch (WalkBatch records with n >= 0) as ONE fused
    launch, then the hidden-state chain through their frames in order.
    Returns (StepOutputs, scenes, h) with h [1, D, H] after the last frame.
    ``cell`` (--use_grid_lstm): the encoder stage in every frame, which makes
    the frames one sequential chain (encoder_step.EncoderChain)."""
    scs = [scene_from_record(r, loader, pairing=pairing) for r in recs]
    if not scs:
        return None, scs, h
    pk = pack(scs, args.rnn_size, nmax=params.nmax)
    S, F = len(scs), pk["F"]
    t = {k: torch.from_numpy(v).to(device) for k, v in pk.items() if isinstance(v, np.ndarray)}
    G = torch.from_numpy(context_G(args.seed, S)).to(device)
    if cell is not None:
        from .encoder_step import EncoderChain
        out, h = EncoderChain(params, cell, lam=args.lambda_param).run(
            t["pos"], t["vislet"], G, t["targets"], t["n_active"], t["n_frames"], h.contiguous(),
            ped_mask=t["ped_mask"], stride=0)
        return out, scs, h
    h0 = torch.zeros((S, fs.HIDDEN_LEN, args.rnn_size), device=device)
    out = fs.step_fused(params, t["pos"], t["vislet"], G, t["targets"], t["n_active"], h0,
                        n_frames=t["n_frames"], ped_mask=t["ped_mask"], stride=0,
                        lam=args.lambda_param, want_attn=True)
    nf = pk["n_frames"]
    if nf.sum() > 0:
        s_idx = torch.from_numpy(np.repeat(np.arange(S), nf)).to(device)
        f_idx = torch.from_numpy(np.concatenate([np.arange(n) for n in nf])).to(device)
        A = out.attn[s_idx, f_idx].unsqueeze(0).contiguous()        # [1, frames, D, D]
        h = fs.frame_recurrence(A, h.contiguous())                  # train.py:240-252, in order
    return out, scs, h


def leg_params(args, device, nmax=NODE_SLICE_NMAX):
    return fs.init_params(nmax, seed=args.seed, device=device)


def training_leg(args, device, params, log=print):
    """train.py:23-365 (mode reference).  Returns per-dataset summary rows
    {d: [(e, b, ADE, FDE, n), ...]} and the final hidden state."""
    datasets = sorted({2, 3, 4, 5} - {args.leaveDataset})            # train.py:38-39
    tlog = TrainLog()
    counters = {"num_targets": 0, "num_end_targets": 0}              # train.py:35-36
    e_done, frame = 0, 1                                              # train.py:29, 34
    h = torch.zeros((1, fs.HIDDEN_LEN, args.rnn_size), device=device)
    cell = encoder_cell(args, device) if getattr(args, "use_grid_lstm", 0) else None
    summary = {}
    for d in datasets:
        try:
            loader = DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=d, sel=0,
                                data_root=args.data_root)           # train.py:50
        except FileNotFoundError as exc:                              # town_center.csv (5) is absent
            log(f"dataset {d}: {exc}")
            continue
        rows = summary.setdefault(d, [])
        epoch, t0 = [], time.time()
        for item in walks.train_walk(loader, args, args.num_epochs, frame=frame,
                                     counters=counters, epoch0=e_done):
            if not isinstance(item, str):
                epoch.append(item)
                continue
            ran = [r for r in epoch if r.n >= 0]
            out, scs, h = launch_records(args, ran, loader, params, device, h, "train_log", cell)
            if out is not None:
                pred = out.pred.cpu().numpy()
                ade, fde = fs.batch_errors(out.metrics, leave_dataset=args.leaveDataset,
                                           num_nodes=[max(r.n, 1) for r in ran])
                for s, r in enumerate(ran):
                    n = r.n
                    if r.n_frames and cell is None:     # the frames of a batch predict alike
                        tlog.add(pred[s, 0, :, :n].reshape(2, fs.PRED_LEN, n), r.n_frames,
                                 r.target_traj)
                    for f in range(r.n_frames if cell is not None else 0):   # they differ
                        tlog.add(pred[s, f, :, :n].reshape(2, fs.PRED_LEN, n), 1, r.target_traj)
                    rows.append((r.index[0], r.index[1], float(ade[s]), float(fde[s]), n))
                    e, b = r.index
                    if (args.save_dir and r.outcome == "next"
                            and checkpoint.save_due(e, b, loader.num_batches, args.save_every)):
                        checkpoint.save_params(checkpoint.checkpoint_prefix(
                            args.save_dir, d, e, b, loader.num_batches), params)   # :330-341
            if args.log_dir:
                tlog.write(args.log_dir, d)                          # :346-351, every epoch
            log(f"dataset {d} epoch {e_done}: {len(ran)} batches in one launch, "
                f"{time.time() - t0:.2f}s")
            e_done += 1
            epoch, t0 = [], time.time()
        frame = counters.get("frame", frame)
        if args.log_dir:
            np.savetxt(os.path.join(args.log_dir, f"g2k_MPC_batch_metrics_kfold_{d}.csv"),
                       np.array(rows, dtype=np.float64).reshape(-1, 5), delimiter=",")
            with open(os.path.join(args.log_dir, f"g2k_lstm_counts_{d}.txt"), "w") as f:  # :361-364
                f.write(f"Dataset {d}= ADE steps {counters['num_targets']}\n"
                        f"FDE steps = {counters['num_end_targets']}")
    return summary, h, counters


def validate(args, device, params, log=print, loader=None, start_pointer=0):
    """The validation leg on dataset l = --leaveDataset (train.py:371-695).
    Returns (cv_ade_err, cv_fde_err) per validation batch with errors.
    ``start_pointer``: the reference's 0 (reset_data_pointer(valid=True),
    :377), or None for the file's first frame (--valid_from_seed)."""
    l = args.leaveDataset
    loader = loader or DataLoader(args, datasets=[0, 1, 2, 3, 4, 5], start=l, sel=0,
                                  data_root=args.data_root)          # :376
    start = loader.seed if start_pointer is None else start_pointer
    recs = []
    gen = walks.valid_walk(loader, args, start_pointer=start)       # fresh graph, frame = 1
    try:
        while True:
            recs.append(next(gen))
    except StopIteration as stop:
        end = stop.value
    ran = [r for r in recs if r.n >= 0]                               # n = -1: the reference raises
    h = torch.zeros((1, fs.HIDDEN_LEN, args.rnn_size), device=device)   # :449
    cell = encoder_cell(args, device) if getattr(args, "use_grid_lstm", 0) else None
    out, scs, h = launch_records(args, ran, loader, params, device, h, "row", cell)
    cv_ade_err, cv_fde_err = [], []
    if out is not None:
        ade, fde = fs.batch_errors(out.metrics, leave_dataset=l,
                                   num_nodes=[max(r.n, 1) for r in ran])   # :668-674
        for s, r in enumerate(ran):
            if r.n > 0 and np.isfinite(ade[s]):                       # :639 num_nodes > 0
                cv_ade_err.append(float(ade[s]))
                cv_fde_err.append(float(fde[s]))
    if end == "crash_n1":
        log("validation: a batch with one node (the reference raises IndexError at train.py:445)")
    log(f"Cross-Validation total mean error (ADE) for dataset {l} = "
        f"{np.mean(cv_ade_err) if cv_ade_err else float('nan')}")
    log(f"Cross-Validation total final error (FDE) for dataset {l} = "
        f"{np.mean(cv_fde_err) if cv_fde_err else float('nan')}")
    if args.save_dir:
        prev = checkpoint.read_state(args.save_dir)
        e = checkpoint.epoch_of(prev) if prev else 0                  # :383-388
        vb = len(recs) - 1 if recs else 0
        prefix = os.path.join(args.save_dir, f"g2k_MPC_model_kfold_val_{l}.ckpt-"
                                             f"{e * loader.valid_num_batches + vb}")
        checkpoint.save_params(prefix, params)                        # :690-693
    return cv_ade_err, cv_fde_err


# ---------------------------------------------------------------------------
# --mode train
# ---------------------------------------------------------------------------
class HipStepper:
    """One rank's train steps on the GPU over its shard of every global step
    (bound once: the shard's scenes gathered into HBM, one g2k_train_step_f32
    plan per step).  ``fused``: gradient and update in one call (one rank);
    ``grad`` + the caller's all-reduce + ``apply`` (g2k_update_f32) across
    ranks."""

    def __init__(self, args, plan, shard_idx, device, steps):
        from .train_step import TrainPlan, flat_params
        sub = plan_subset(plan, shard_idx)
        t = sub.to_device(device)
        S = sub.S
        per = S // steps
        G = torch.from_numpy(context_G(args.seed, S)).to(device)
        h0 = torch.zeros((S, fs.HIDDEN_LEN, args.rnn_size), device=device)
        loss = getattr(args, "loss", "l2")
        self.flat, p = flat_params(fs.init_params(plan.Nmax, seed=args.seed, device=device), loss)
        self.ms = torch.ones_like(self.flat)          # TF RMSProp's "rms" slot starts at 1
        self.kw = dict(lr=args.learning_rate, decay=args.decay_rate, grad_clip=args.grad_clip)
        sl = lambda k, x: x[k * per:(k + 1) * per]                    # noqa: E731
        self.plans = [TrainPlan(p, sl(k, t["pos"]), sl(k, t["vislet"]), sl(k, G),
                                sl(k, t["targets"]), sl(k, t["n_active"]), sl(k, h0),
                                n_frames=sl(k, t["n_frames"]), ped_mask=sl(k, t["ped_mask"]),
                                stride=0, lam=args.lambda_param, loss=loss) for k in range(steps)]
        self._keep = (t, G, h0, p)

    def fused(self, k):
        return self.plans[k].run(self.flat, self.ms, **self.kw)

    def grad(self, k):
        return self.plans[k].run()

    def apply(self, g):
        from .train_step import optimizer_update
        optimizer_update(self.flat, g, ms=self.ms, **self.kw)

    def params(self):
        return self.flat.detach().double().cpu().numpy()


def plan_subset(plan, idx):
    """The scenes ``idx`` of a RealPlan (same datasets and columns)."""
    from dataclasses import replace
    idx = np.asarray(idx, dtype=np.int64)
    return replace(plan, names=[plan.names[i] for i in idx], pointers=plan.pointers[idx],
                   pos_col=plan.pos_col[idx], tgt_col=plan.tgt_col[idx],
                   n_active=plan.n_active[idx], n_frames=plan.n_frames[idx],
                   vis_off=plan.vis_off[idx])


def shard_schedule(total, batch, rank, world):
    """(steps, this rank's scene indices, step-major): global step k takes
    scenes [k*batch, (k+1)*batch) and rank r its contiguous shard of them."""
    from .dist import shard_scenes
    steps = total // batch
    if steps < 1:
        raise ValueError(f"{total} scenes < one global batch of {batch}")
    lo, hi = shard_scenes(batch, rank, world)
    if any(shard_scenes(batch, r, world)[1] - shard_scenes(batch, r, world)[0] != hi - lo
           for r in range(world)):
        raise ValueError(f"--train_batch {batch} must be a multiple of the world size {world}")
    idx = np.concatenate([np.arange(k * batch + lo, k * batch + hi) for k in range(steps)])
    return steps, idx


def train_mode(args, plan, device, *, rank=0, world=1, group=None, stepper_cls=None, log=print):
    """--mode train over a RealPlan: num_epochs passes of `steps` global steps.
    Returns (final flat parameters (float64, host), per-step loss per
    prediction)."""
    from .dist import allreduce_grad
    steps, idx = shard_schedule(plan.S, args.train_batch, rank, world)
    stepper = (stepper_cls or HipStepper)(args, plan, idx, device, steps)
    losses = []
    lbuf = None                  # per-step (loss, count), kept where the gradient lives
    for e in range(args.num_epochs):
        t0 = time.time()
        for k in range(steps):
            if world == 1:
                g = stepper.fused(k)                 # nothing to all-reduce: update in the call
            else:
                g = stepper.grad(k)                  # this rank's shard
                allreduce_grad(g, group)             # ONE collective per step
                stepper.apply(g)                     # the same update on every rank
            if lbuf is None:
                lbuf = torch.empty((steps, 2), dtype=g.dtype, device=g.device)
            lbuf[k].copy_(g[-2:])                    # stream-ordered: no host round trip per step
        gl = lbuf.double().tolist()                  # ONE host read per epoch
        losses += [float(a / max(c, 1.0)) for a, c in gl]
        if rank == 0:
            log(f"train epoch {e}: {steps} steps x {args.train_batch} scenes "
                f"({world} rank(s)), loss/prediction {losses[-1]:.6g}, {time.time() - t0:.2f}s")
    return stepper.params(), losses


def train(args, log=print):
    device = torch.device(args.device)
    if args.log_dir:
        os.makedirs(args.log_dir, exist_ok=True)
    if args.mode == "train":
        return run_train_mode(args, device, log=log)
    params = leg_params(args, device)
    training_leg(args, device, params, log=log)
    try:
        validate(args, device, params, log=log,
                 start_pointer=None if getattr(args, "valid_from_seed", 0) else 0)
    except FileNotFoundError as exc:
        log(f"validation dataset {args.leaveDataset}: {exc}")


def run_train_mode(args, device, log=print):
    """--mode train under torchrun (WORLD_SIZE / RANK / LOCAL_RANK) or alone."""
    from . import realdata as rd
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.world_size and args.world_size != world:
        raise SystemExit(f"--world_size {args.world_size} but WORLD_SIZE={world}")
    group = None
    if world > 1:
        import torch.distributed as dist
        if device.type == "cuda":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    names = [n for n in rd.fold_datasets(args.leaveDataset)]
    raw = rd.load_raw(names, args.data_root)
    plan = rd.plan_scenes(args.train_scenes or rd.count_scenes(raw, args.n_max), raw,
                          nmax=args.n_max or None)
    params, losses = train_mode(args, plan, device, rank=rank, world=world, group=group, log=log)
    if rank == 0 and args.save_dir:
        flat = torch.from_numpy(params.astype(np.float32))
        from .train_step import GRAD_ORDER
        keys = GRAD_ORDER + (("head",) if args.loss == "nll" else ())
        shapes = {k: tuple(getattr(fs.init_params(plan.Nmax), k).shape) for k in GRAD_ORDER}
        shapes["head"] = (3, fs.PRED_LEN)
        views, o = {}, 0
        for k in keys:
            n = int(np.prod(shapes[k]))
            views[k] = flat[o:o + n].view(shapes[k])
            o += n
        checkpoint.save_params(os.path.join(args.save_dir, "g2k_MPC_model_train_mode.ckpt-"
                                            f"{args.num_epochs}"), fs.G2KParams(**views))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return params, losses


def main(argv=None):
    args = ArgsParser().parser.parse_args(argv)
    train(args)


if __name__ == '__main__':
    main()
