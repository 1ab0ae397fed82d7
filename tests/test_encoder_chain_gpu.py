"""GPU: --use_grid_lstm's encoder chain as ONE workgroup walking the frames
(g2k_encoder_chain_f32, ABI 8; multimodaltraj_2_amd/encoder_step.py) against
the same three bodies as three launches per frame issued from a Python loop
(the round-4 form): bit-identical pred, attn, cost and hidden state, and the
time per frame of each.  Parity of the chain against the oracle is
tests/test_train_legs_gpu.py::test_training_leg_with_grid_lstm_encoder."""
import json
import time

import numpy as np
import pytest
import torch

from multimodaltraj_2_amd import frame_step as fs
from multimodaltraj_2_amd.encoder_step import EncoderChain
from multimodaltraj_2_amd.helper import gridlstm, neighborhood_vis_loc_encoder
from multimodaltraj_2_amd.synthetic import make_batch

pytestmark = pytest.mark.gpu


def python_loop(params, cell, pos, vislet, G, n_active, n_frames, h, F, lam=fs.LAMBDA):
    """The chain as round 4 ran it: three Python-issued launches per frame."""
    S, Nmax, D = int(pos.shape[0]), int(pos.shape[2]), fs.HIDDEN_LEN
    dev = pos.device
    X, Rel = fs.frame_embed(params, pos, vislet, n_active, F, stride=0)
    Xe = X.clone()
    pred = torch.zeros((S, F, 2 * fs.PRED_LEN, Nmax), device=dev)
    attn = torch.zeros((S, F, D, D), device=dev)
    cost = torch.zeros((S, F, fs.OBS_LEN, fs.OBS_LEN), device=dev)
    scratch = torch.empty((D, D), device=dev)
    nf = n_frames.cpu().numpy()
    for s in range(S):
        for f in range(int(nf[s])):
            gridlstm(X[s, f, :D], h[0], cell.W, cell.b, cell.peep, feature_size=cell.feature_size,
                     num_units=cell.num_units, out=Xe[s, f, :D], state_out=scratch)
            fs.mcr_forward(params, Xe[s, f:f + 1], Rel[s:s + 1], G[s:s + 1], n_active[s:s + 1],
                           lam=lam, out=(attn[s, f:f + 1], cost[s, f:f + 1], pred[s, f:f + 1]))
            fs.frame_recurrence(attn[s:s + 1, f:f + 1], h)
    return pred, attn, cost, h


def setup(gpu, S, F, H=128, Nmax=32, seed=5):
    b = make_batch(S, Nmax, H, F=F, seed=seed)
    t = b.to_device(gpu)
    n_frames = torch.tensor([F - (s % 3) for s in range(S)], dtype=torch.int32, device=gpu)
    G = torch.from_numpy(np.random.default_rng(seed).standard_normal((S, 16, 8)).astype(np.float32)).to(gpu)
    params = fs.init_params(Nmax, seed=1, device=gpu)
    cell = neighborhood_vis_loc_encoder(hidden_size=H, hidden_len=16, num_layers=2, grid_size=4,
                                        embedding_size=64, device=gpu, seed=3).rnn
    h0 = torch.from_numpy(np.random.default_rng(seed + 1).standard_normal((1, 16, H)).astype(np.float32)).to(gpu)
    return t, n_frames, G, params, cell, h0


@pytest.mark.parametrize("H", [64, 128, 256, 512])
def test_chain_entry_bit_identical_to_python_loop(gpu, H):
    S, F = 5, 7
    t, n_frames, G, params, cell, h0 = setup(gpu, S, F, H=H)
    n_frames[2] = 0                                   # a batch without frames: skipped
    h_c, h_p = h0.clone(), h0.clone()
    out, _ = EncoderChain(params, cell).run(t["pos"], t["vislet"], G, t["targets"], t["n_active"],
                                            n_frames, h_c, stride=0)
    pred, attn, cost, _ = python_loop(params, cell, t["pos"], t["vislet"], G, t["n_active"],
                                      n_frames, h_p, F)
    torch.cuda.synchronize()
    for a, b in ((out.pred, pred), (out.attn, attn), (out.cost, cost), (h_c, h_p)):
        assert torch.equal(a, b)
    assert float(h_c.abs().sum()) > 0 and not torch.equal(h_c, h0)


def test_chain_entry_time_per_frame(gpu):
    """The one-workgroup chain against the Python loop of launches over the
    same 160 frames (timing printed; the chain kernel must not be slower).
    Wall time per frame including the entry point's host work and its
    embed / error launches: 12.2 us in round 5 (global hand-offs between
    barriers), 3.4 us with every hand-off in LDS (profiles/r11e_chain_stamps.txt);
    the bound below is a regression guard with room for box-to-box spread."""
    S, F = 8, 20
    t, n_frames, G, params, cell, h0 = setup(gpu, S, F)
    n_frames = torch.full((S,), F, dtype=torch.int32, device=gpu)
    chain = EncoderChain(params, cell)

    def c_run():
        h = h0.clone()
        chain.run(t["pos"], t["vislet"], G, t["targets"], t["n_active"], n_frames, h, stride=0)

    def py_run():
        h = h0.clone()
        python_loop(params, cell, t["pos"], t["vislet"], G, t["n_active"], n_frames, h, F)

    res = {}
    for name, fn in (("chain_kernel", c_run), ("python_loop", py_run)):
        fn()
        torch.cuda.synchronize()
        best = float("inf")
        for _ in range(3):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        res[name] = best / (S * F) * 1e6
    print(json.dumps({"us_per_frame": res, "frames": S * F}))
    assert res["chain_kernel"] <= res["python_loop"]
    assert res["chain_kernel"] <= 6.0
