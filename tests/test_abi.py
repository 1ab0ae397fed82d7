"""The C-ABI library loads, exports every symbol include/g2k_hip.h declares,
and rejects bad arguments before touching the GPU (runs on CPU)."""
import ctypes
import os
import re

import pytest

from multimodaltraj_2_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "g2k_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(g2k_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert sorted(_lib.SYMBOLS) == declared_functions()


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.g2k_abi_version() == _lib.ABI_VERSION


def _dims(**kw):
    d = dict(S=2, F=20, T=8, L=12, D=16, H=128, Nmax=32, W=27, stride=1)
    d.update(kw)
    return _lib.G2KDims(**d)


@pytest.mark.parametrize("bad,code", [(dict(T=10), -4), (dict(D=10), -4), (dict(H=96), -4),
                                      (dict(H=384), -4),
                                      (dict(Nmax=0), -1), (dict(Nmax=300), -1), (dict(W=26), -1),
                                      (dict(stride=-1), -1), (dict(S=-1), -1)])
def test_step_rejects_bad_geometry(bad, code):
    lib = _lib.load()
    w = _lib.G2KWeights(*([ctypes.c_void_p(16)] * 7))
    p = ctypes.c_void_p(16)
    rc = lib.g2k_step_fused_f32(ctypes.byref(_dims(**bad)), ctypes.byref(w), p, p, p, p, p, None,
                                None, p, p, p, p, None, None, 5e-4, p, 1 << 30, None)
    assert rc == code
    assert lib.g2k_last_error()


def _split(x):
    return x << _lib.STEP_SPLIT_SHIFT


def test_step_rejects_null_and_sizes_the_split_workspace():
    lib = _lib.load()
    w = _lib.G2KWeights(*([ctypes.c_void_p(16)] * 7))
    p = ctypes.c_void_p(16)
    rc = lib.g2k_step_fused_f32(ctypes.byref(_dims()), ctypes.byref(w), None, p, p, p, p, None,
                                None, p, p, p, p, None, None, 5e-4, p, 1 << 30, None)
    assert rc == -1
    # one workgroup per scene (S >= 256 CUs, or G2K_STEP_SPLIT(1)): every
    # intermediate stays on chip
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims(S=256))) == 0
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims(flags=_split(1)))) == 0
    # split scenes: one 64-byte ticket line per 16 scenes + [S][X][8] partials
    # (S = 2: automatic X = min(4, 256 / S) = 4; S = 128: X = 2)
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims())) == 64 + 2 * 4 * 8 * 4
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims(S=128))) == 8 * 64 + 128 * 2 * 8 * 4
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims(flags=_split(2)))) == 64 + 2 * 2 * 8 * 4
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims(F=1))) == 0     # one frame: X = 1
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims(T=9))) == -1
    assert 0 < lib.g2k_step_lds_bytes(ctypes.byref(_dims())) <= 160 * 1024
    # the split must name 0..4 workgroups, and X > 1 needs its workspace
    assert lib.g2k_step_workspace_bytes(ctypes.byref(_dims(flags=_split(5)))) == -1
    rc = lib.g2k_step_fused_f32(ctypes.byref(_dims(flags=_split(5))), ctypes.byref(w), p, p, p, p,
                                p, None, None, p, p, p, p, None, None, 5e-4, p, 1 << 30, None)
    assert rc == -1
    rc = lib.g2k_step_fused_f32(ctypes.byref(_dims()), ctypes.byref(w), p, p, p, p, p, None,
                                None, p, p, p, p, None, None, 5e-4, None, 0, None)
    assert rc == -1 and b"workspace" in lib.g2k_last_error()


def test_other_entry_points_validate():
    lib = _lib.load()
    p = ctypes.c_void_p(16)
    assert lib.g2k_frame_recurrence_f32(ctypes.byref(_dims(H=100)), p, p, 3, None) == -4
    assert lib.g2k_ade_fde_f32(ctypes.byref(_dims(L=10)), p, p, p, None, None, 0, p, None) == -4
    assert lib.g2k_ade_fde_f32(ctypes.byref(_dims()), p, p, p, None, None, 7, p, None) == -1
    assert lib.g2k_infer_rlns_f32(None, p, 4, 4, None) == -1
    assert lib.g2k_eval_rln_ngh_f32(p, p, 4, 0, None) == -1
    assert lib.g2k_step_lds_bytes(ctypes.byref(_dims(T=9))) == 0


def test_zero_scenes_is_a_noop():
    lib = _lib.load()
    w = _lib.G2KWeights(*([ctypes.c_void_p(16)] * 7))
    p = ctypes.c_void_p(16)
    rc = lib.g2k_step_fused_f32(ctypes.byref(_dims(S=0)), ctypes.byref(w), p, p, p, p, p, None,
                                None, p, p, p, p, None, None, 5e-4, p, 0, None)
    assert rc == 0


def test_gridlstm_and_train_entry_points_validate():
    lib = _lib.load()
    p = ctypes.c_void_p(16)
    # g2k_gridlstm_f32(in, ld_in, state, ld_state, W, b, peep, out, state_out, rows, K, fs, u, s)
    assert lib.g2k_gridlstm_f32(None, 16, p, 16, p, p, None, p, p, 4, 4, 4, 2, None) == -1
    assert lib.g2k_gridlstm_f32(p, 15, p, 16, p, p, None, p, p, 4, 4, 4, 2, None) == -1
    assert lib.g2k_gridlstm_f32(p, 16, p, 24, p, p, None, p, p, 4, 4, 4, 3, None) == -4
    # state_out aliases state with a wider pitch
    assert lib.g2k_gridlstm_f32(p, 16, p, 20, p, p, None, p, p, 4, 4, 4, 2, None) == -1
    assert lib.g2k_gridlstm_f32(p, 16, p, 16, p, p, None, p, p, 0, 4, 4, 2, None) == 0
    d = _dims()
    assert lib.g2k_grad_size(ctypes.byref(d)) == 24 * 32 + 496
    need = lib.g2k_grad_workspace_bytes(ctypes.byref(d))
    # one gradient row [P + 2] per workgroup (S X of them, the fused kernel's
    # output), the 64-byte line of the folded update's ticket, then the split
    # workspace (scene tickets, metric partials)
    assert need == 2 * 4 * (24 * 32 + 498) * 4 + 64 + 64 + 2 * 4 * 8 * 4
    one = lib.g2k_grad_workspace_bytes(ctypes.byref(_dims(flags=_split(1))))
    assert one == 2 * (24 * 32 + 498) * 4 + 64
    assert lib.g2k_train_workspace_bytes(ctypes.byref(d)) == need
    w = _lib.G2KWeights(*([p] * 7))
    rc = lib.g2k_step_grad_f32(ctypes.byref(d), ctypes.byref(w), p, p, p, p, p, None, None, 5e-4,
                               p, p, need - 4, None)
    assert rc == -1 and b"workspace" in lib.g2k_last_error()
    rc = lib.g2k_step_grad_f32(ctypes.byref(_dims(T=9)), ctypes.byref(w), p, p, p, p, p, None,
                               None, 5e-4, p, p, need, None)
    assert rc == -4
    assert lib.g2k_update_f32(None, None, p, 10, 0.1, 0.9, 10.0, None) == -1
    # the one-rank fused gradient + update: NULL params, short workspace
    rc = lib.g2k_step_grad_update_f32(ctypes.byref(d), ctypes.byref(w), p, p, p, p, p, None, None,
                                      5e-4, p, p, need, None, None, 5e-3, 0.95, 10.0, None)
    assert rc == -1 and b"params" in lib.g2k_last_error()
    rc = lib.g2k_step_grad_update_f32(ctypes.byref(d), ctypes.byref(w), p, p, p, p, p, None, None,
                                      5e-4, p, p, need - 4, p, None, 5e-3, 0.95, 10.0, None)
    assert rc == -1 and b"workspace" in lib.g2k_last_error()
    assert lib.g2k_update_f32(p, None, p, 0, 0.1, 0.9, 10.0, None) == 0
    # g2k_train_step_f32(d, w, pos, vis, G, tgt, nact, nfr, mask, h_in, h_out, pred, met, lam,
    #                    grad, ws, ws_bytes, params, ms, lr, decay, clip, stream)
    rc = lib.g2k_train_step_f32(ctypes.byref(d), ctypes.byref(w), p, p, p, p, p, None, None, p, p,
                                p, p, 5e-4, p, p, need - 4, None, None, 5e-3, 0.95, 10.0, None)
    assert rc == -1 and b"workspace" in lib.g2k_last_error()
    rc = lib.g2k_train_step_f32(ctypes.byref(d), ctypes.byref(w), p, p, p, p, p, None, None, None,
                                p, p, p, 5e-4, p, p, need, None, None, 5e-3, 0.95, 10.0, None)
    assert rc == -1
    rc = lib.g2k_train_step_f32(ctypes.byref(_dims(H=96)), ctypes.byref(w), p, p, p, p, p, None,
                                None, p, p, p, p, 5e-4, p, p, need, None, None, 5e-3, 0.95, 10.0,
                                None)
    assert rc == -4


def test_small_D_entry_points():
    """D in 1..16 for the class-level forward, the recurrence and the errors
    (sample.py's num_freq_blocks = 10); the fused step needs D = 16."""
    lib = _lib.load()
    p = ctypes.c_void_p(16)
    w = _lib.G2KWeights(*([p] * 7))
    assert lib.g2k_frame_recurrence_f32(ctypes.byref(_dims(D=17)), p, p, 3, None) == -4
    assert lib.g2k_frame_recurrence_f32(ctypes.byref(_dims(D=10, S=0)), p, p, 3, None) == 0
    assert lib.g2k_mcr_forward_f32(ctypes.byref(_dims(D=0)), ctypes.byref(w), p, p, p, p, p, p, p,
                                   5e-4, None) == -4
    assert lib.g2k_mcr_forward_f32(ctypes.byref(_dims(D=10, S=0)), ctypes.byref(w), p, p, p, p, p,
                                   p, p, 5e-4, None) == 0


def test_context_conv_validates():
    lib = _lib.load()
    p = ctypes.c_void_p(16)
    assert lib.g2k_context_conv_workspace_bytes(576, 720, 16) == (576 + 3 - 16) * 256 * 4
    assert lib.g2k_context_conv_workspace_bytes(10, 10, 16) == -1
    assert lib.g2k_context_conv_f32(p, 576, 720, 5, p, 16, 5e-4, p, None, p, 1 << 30, None) == -4
    assert lib.g2k_context_conv_f32(p, 576, 720, 3, p, 16, 5e-4, None, None, p, 1 << 30, None) == -1
    assert lib.g2k_context_conv_f32(p, 576, 720, 3, p, 16, 5e-4, p, None, p, 16, None) == -1


def test_encoder_chain_validates():
    """g2k_encoder_chain_f32 (ABI 8) rejects bad arguments before any device
    call; zero frames are a no-op."""
    lib = _lib.load()
    w = _lib.G2KWeights(*([ctypes.c_void_p(16)] * 7))
    p = ctypes.c_void_p(16)

    def call(d, fs=4, u=2, **null):
        a = dict(X=p, Rel=p, G=p, na=p, nf=p, W=p, b=p, peep=None, Xe=p, cs=p, attn=p, cost=p,
                 pred=p, h=p)
        a.update(null)
        return lib.g2k_encoder_chain_f32(ctypes.byref(d), ctypes.byref(w), a["X"], a["Rel"], a["G"],
                                         a["na"], a["nf"], a["W"], a["b"], a["peep"], fs, u, a["Xe"],
                                         a["cs"], a["attn"], a["cost"], a["pred"], a["h"], 0.0005,
                                         None)
    assert call(_dims(S=0)) == 0                          # nothing to run
    assert call(_dims(F=0)) == 0
    assert call(_dims(H=96)) == -4                        # unsupported hidden size
    assert call(_dims(D=10)) == -4                        # the chain needs D = 16
    assert call(_dims(), fs=4, u=1) == -4                 # feature_size must be 2 num_units
    assert call(_dims(), fs=8, u=3) == -4
    assert call(_dims(), h=None) == -1                    # required buffers
    assert call(_dims(), nf=None) == -1
    assert call(_dims(), h=ctypes.c_void_p(20)) == -1     # h 16-byte aligned
    assert lib.g2k_last_error()


def test_split_sizing_without_a_gpu_is_explicit():
    """ABI 9: the automatic split for a given CU count is host arithmetic
    (g2k_step_split_for_cus, no HIP call), and an explicit split makes the
    workspace size independent of any device (include/g2k_hip.h)."""
    import ctypes

    from multimodaltraj_2_amd import frame_step as fs
    lib = _lib.load()
    assert fs.split_for_cus(256, 20, cus=256) == 1
    assert fs.split_for_cus(128, 20, cus=256) == 2
    assert fs.split_for_cus(128, 20, cus=304) == 2
    assert fs.split_for_cus(64, 20, cus=256) == 4
    assert fs.split_for_cus(16, 20, cus=256) == 4          # at most kMaxSplit
    assert fs.split_for_cus(16, 3, cus=256) == 3           # at most F
    assert fs.split_for_cus(100, 20, cus=80) == 1
    assert fs.split_for_cus(128, 20, split=3, cus=256) == 3          # the request
    assert fs.split_for_cus(128, 20, coresident=True, cus=256) == 1  # launches in flight
    # loop-invariant launches (stride 0, shared targets; L2, Nmax <= 85): one frame's work
    inv = dict(stride=0, targets_shared=True, Nmax=32)
    assert fs.split_for_cus(128, 20, cus=256, **inv) == 1
    assert fs.split_for_cus(128, 20, split=2, cus=256, **inv) == 2          # the request stands
    assert fs.split_for_cus(128, 20, cus=256, stride=0, targets_shared=False, Nmax=32) == 2
    assert fs.split_for_cus(128, 20, cus=256, stride=1, targets_shared=True, Nmax=32) == 2
    assert fs.split_for_cus(128, 20, cus=256, stride=0, targets_shared=True, Nmax=128) == 2
    assert fs.split_for_cus(128, 20, cus=256, loss="nll", **inv) == 2
    d = _lib.G2KDims(128, 20, 8, 12, 16, 128, 32, 27, 1, 0)
    assert lib.g2k_step_split_for_cus(ctypes.byref(d), 0) == -1
    sizes = set()
    for x in (1, 2, 4):
        d = _lib.G2KDims(128, 20, 8, 12, 16, 128, 32, 27, 1, fs.step_flags(split=x))
        nb = lib.g2k_step_workspace_bytes(ctypes.byref(d))
        assert nb == (0 if x == 1 else (128 + 15) // 16 * 64 + 128 * x * 8 * 4)
        sizes.add(nb)
        tb = lib.g2k_train_workspace_bytes(ctypes.byref(d))
        P = lib.g2k_grad_size(ctypes.byref(d))
        assert tb == 128 * x * (P + 2) * 4 + 64 + nb       # one gradient row per workgroup
    assert len(sizes) == 3


def test_loop_invariant_launches_hold_one_ring_slot():
    """Stride 0 with shared targets and one workgroup per scene
    (g2k_scene.hip frames_invariant): the forward forms one head per chunk,
    so its rings hold one slot — a smaller LDS carve-up than the same launch
    with per-frame targets, whose rings hold every frame of the chunk; train
    mode and split launches keep the general layout (host arithmetic, no
    GPU)."""
    from multimodaltraj_2_amd import frame_step as fs
    lib = _lib.load()

    def lds(F, shared, split, coresident=False, stride=0, W=8):
        d = _lib.G2KDims(128, F, 8, 12, 16, 128, 32, W, stride,
                         fs.step_flags(targets_shared=shared, split=split, coresident=coresident))
        return lib.g2k_step_lds_bytes(ctypes.byref(d))

    general, inv = lds(29, False, 1), lds(29, True, 1)
    assert general - inv == (29 - 1) * (16 * 16 + 24 * 8) * 4       # As and M slots
    assert lds(29, False, 1, coresident=True) - lds(29, True, 1, coresident=True) == general - inv
    assert lds(29, True, 2) == lds(29, False, 2)                     # split: general path
    assert lds(20, True, 1, stride=1, W=27) == lds(20, False, 1, stride=1, W=27)
    assert fs.step_coresidency(128, 29, 128, 32, 8, 0, True, True) == 2
