"""Workgroup timelines of the scene kernel (development probe, not product
code): a copy of csrc with s_memtime stamps at the phase boundaries of every
workgroup, the CU it ran on (HW_ID / XCC_ID) and the launch it belongs to,
built into tools/ab/libg2k_timeline.so on the CPU host; on the GPU box it
runs launches one at a time (one stream) and concurrently (round-robin over
several streams) and prints per-launch phase times and how many workgroups
shared a CU at once.

usage: python tools/probes/wg_timeline.py --build
       python tools/probes/wg_timeline.py CONFIG [STREAMS [SPLIT [on|off]]]   (on: G2K_STEP_CORESIDENT)"""
import ctypes
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
OUT = os.environ.get("TL_OUT", os.path.join(ROOT, "tools", "ab", "libg2k_timeline.so"))
NREC = 128

DEF = r"""
__device__ unsigned g2k_tl_buf[8192 * 128];
__device__ unsigned g2k_tl_ctr;
// stamps go to a per-workgroup LDS record (no global round trip on the
// stamped path); the last wave to exit copies the record to g2k_tl_buf
#define G2K_TL(k, cond) do { if ((cond) && c.lane == 0) { \
  reinterpret_cast<unsigned*>(c.sWi - lay.o_wi + lay.total)[(k)] = (unsigned)__builtin_amdgcn_s_memtime(); } } while (0)
"""
EXPORT = r"""
extern "C" int g2k_tl_copy(unsigned* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g2k::g2k_tl_buf), (size_t)n * 4, 0, hipMemcpyDeviceToHost);
}
extern "C" int g2k_tl_count(unsigned* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g2k::g2k_tl_ctr), 4, 0, hipMemcpyDeviceToHost);
}
extern "C" int g2k_tl_reset(void) {
  static unsigned z = 0;
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g2k::g2k_tl_ctr), &z, 4, 0, hipMemcpyHostToDevice);
}
"""
ENTRY = r"""  if (c.wv == 0) {
    unsigned* r = reinterpret_cast<unsigned*>(smem + lay.total);
    const unsigned t0 = (unsigned)__builtin_amdgcn_s_memtime();
    for (int k = c.lane; k < 128; k += 64) r[k] = 0u;
    if (c.lane == 0) {
      r[0] = blockIdx.x + 1;
      r[1] = (unsigned)((uintptr_t)a.h_out >> 8);
      r[2] = __builtin_amdgcn_s_getreg(63492);
      r[3] = __builtin_amdgcn_s_getreg(63508);
      r[4] = t0;
      r[70] = g2k_t_entry;
    }
  }
"""
EXIT = r"""  G2K_TL(32 + c.wv, true);
  if (c.lane == 0) {
    unsigned* r = reinterpret_cast<unsigned*>(smem + lay.total);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    const unsigned old = atomicAdd(r + 127, 1u);
    if (old == (unsigned)(NT / 64 - 1)) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const unsigned s_ = atomicAdd(&g2k_tl_ctr, 1u) & 8191u;   // (wraps: warm-up launches)
      for (int k = 0; k < 127; ++k) g2k_tl_buf[(size_t)s_ * 128 + k] = r[k];
    }
  }
}"""
REPS = [
    ("  extern __shared__ __attribute__((aligned(16))) float smem[];\n",
     "  extern __shared__ __attribute__((aligned(16))) float smem[];\n"
     "  const unsigned g2k_t_entry = (unsigned)__builtin_amdgcn_s_memtime();\n"),
    ("namespace g2k {\nnamespace {\n\nconstexpr int kSceneChunk",
     "namespace g2k {\n" + DEF + "namespace {\n\nconstexpr int kSceneChunk"),
    ("  const size_t lds = (size_t)l.total * 4;", "  const size_t lds = (size_t)l.total * 4 + 512;   // + the LDS stamp record"),
    ("  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;",
     ENTRY + "  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;"),
    ("  // the first frames' attention weights (E -> A -> As into the ring, the",
     "  G2K_TL(5, c.wv == 0);\n  // the first frames' attention weights (E -> A -> As into the ring, the"),
    ("      float4 b0, b1;\n      int f0 = read_as(",
     "      G2K_TL(6, c.wv == 0 && fb == 0);\n      float4 b0, b1;\n      int f0 = read_as("),
    ("  rc.store(a.h_out + (size_t)c.s * kD * H", "  G2K_TL(7, c.wv == 0);\n  rc.store(a.h_out + (size_t)c.s * kD * H"),
    ("    // phase 2 — predictions and errors (GRAD: and the gradient)",
     "    G2K_TL(8 + pw, fb == 0);\n    // phase 2 — predictions and errors (GRAD: and the gradient)"),
    ("  if (NLL) nll_worker_reduce(c, pw);\n  publish_metrics(a, c, pw,",
     "  G2K_TL(20 + pw, true);\n  if (NLL) nll_worker_reduce(c, pw);\n  publish_metrics(a, c, pw,"),
    ("  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");   // no LDS-DMA outlives the workgroup\n}",
     "  asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");   // no LDS-DMA outlives the workgroup\n" + EXIT),
    ("    for (int i = pw; i < nh; i += NP) {",
     "    G2K_TL(48, pw == 0 && fb == 0);\n    int g2k_hk = 0;\n    for (int i = pw; i < nh; i += NP) {"),
    ("        if (lane == 0) lds_store_flag(c.sMflag + fl, f + 1);\n      }\n      __builtin_amdgcn_s_setprio(0);\n    }",
     "        if (lane == 0) lds_store_flag(c.sMflag + fl, f + 1);\n      }\n      __builtin_amdgcn_s_setprio(0);\n"
     "      G2K_TL(49 + (g2k_hk < 6 ? g2k_hk : 6), pw == 0 && fb == 0);\n      ++g2k_hk;\n    }"),
]
STAGE = [
    ("  __builtin_amdgcn_s_barrier();                                 // B1: window + weights landed\n",
     "  G2K_TL(96 + c.wv, fb == 0);\n"
     "  __builtin_amdgcn_s_barrier();                                 // B1: window + weights landed\n"
     "  G2K_TL(56 + (c.wv < kRecW ? 0 : 1), (c.wv == 0 || c.wv == kRecW) && fb == 0);\n"),
    ("  __builtin_amdgcn_s_waitcnt(0xc07f);                           // lgkmcnt(0)\n  __builtin_amdgcn_s_barrier();                                 // B2: V, VG, K1, K2",
     "  G2K_TL(58 + (c.wv < kRecW ? 0 : 1), (c.wv == 0 || c.wv == kRecW) && fb == 0);\n"
     "  G2K_TL(24 + (c.wv - kRecW) % 8, c.wv >= kRecW && c.wv < kRecW + 4 && fb == 0);\n"
     "  __builtin_amdgcn_s_waitcnt(0xc07f);                           // lgkmcnt(0)\n"
     "  G2K_TL(80 + c.wv, fb == 0);\n"
     "  __builtin_amdgcn_s_barrier();                                 // B2: V, VG, K1, K2"),
]
PROLOGUE = [
    ("    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first\n",
     "    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first\n"
     "    G2K_TL(60, c.wv == 0);\n"),
    ("    if (c.tid < lay.fc) {                                // flags hold (global frame + 1)",
     "    G2K_TL(61, c.wv == 0);\n    if (c.tid < lay.fc) {                                // flags hold (global frame + 1)"),
    ("    scalars();\n    scene_recurrence<TPW, NP, CR, !GRAD, INV>(a, lay, c);",
     "    scalars();\n    G2K_TL(62, c.wv == 0);\n    scene_recurrence<TPW, NP, CR, !GRAD, INV>(a, lay, c);"),
    ("  __builtin_amdgcn_s_waitcnt(0x0070);                           // vmcnt(0) lgkmcnt(0)\n",
     "  __builtin_amdgcn_s_waitcnt(0x0070);                           // vmcnt(0) lgkmcnt(0)\n"
     "  G2K_TL(63, (c.wv == 0 || c.wv == kRecW) && fb == 0);\n"),
]
TRAIN = [
    ("      // every worker done with the chunk's frames -> its dU rows into dV\n",
     "      G2K_TL(44, pw == 0 && fb == 0);\n      // every worker done with the chunk's frames -> its dU rows into dV\n"),
    ("      if (ntact > 0) grad_chunk_flush(a, lay, c, fb, cnt, NP);   // (no active pedestrian: all zero)",
     "      G2K_TL(45, pw == 0 && fb == 0);\n      if (ntact > 0) grad_chunk_flush(a, lay, c, fb, cnt, NP);   // (no active pedestrian: all zero)"),
    ("  grad_priv_sum(c, NP);                                // then all producers see sGAcc",
     "  G2K_TL(46, pw == 0);\n  grad_priv_sum(c, NP);                                // then all producers see sGAcc"),
    ("  // the small blocks and dWo, entry by entry over the lanes of the producers",
     "  G2K_TL(47, pw == 0);\n  // the small blocks and dWo, entry by entry over the lanes of the producers"),
]
TRAIN += [
    ("      if (ntact > 0) grad_chunk_flush(a, lay, c, fb, cnt, NP);   // (no active pedestrian: all zero)\n",
     "      if (ntact > 0) grad_chunk_flush(a, lay, c, fb, cnt, NP);   // (no active pedestrian: all zero)\n"
     "      G2K_TL(64, pw == 0 && fb == 0);\n"),
    ("  poll_word(c.sTicket, NP + kRecW);\n", "  G2K_TL(65, pw == 0);\n  poll_word(c.sTicket, NP + kRecW);\n"),
    ("  poll_word(c.sGseq + 1, NP);\n", "  poll_word(c.sGseq + 1, NP);\n  G2K_TL(66, pw == 0);\n"),
    ("      if (c.lane == 0) atomicAdd(c.sGseq, 1);\n    }\n  }\n  if (NLL) nll_worker_reduce(c, NP + c.wv);",
     "      G2K_TL(67, c.wv == 0);\n      if (c.lane == 0) atomicAdd(c.sGseq, 1);\n    }\n  }\n"
     "  if (NLL) nll_worker_reduce(c, NP + c.wv);"),
]
REPS += STAGE + PROLOGUE + TRAIN
# TL_WARM=1 (build): the first vtile / kmats task of a producer run twice,
# stamped around each run (is the first run's time the code's first fetch?)
WARM = [
    ("      if (task < ntile) {\n        scene_vtile(a, lay, c, 16 * task, wcc);\n      } else {\n        scene_kmats(c);",
     "      if (task < ntile) {\n        G2K_TL(112 + 3 * task, fb == 0);\n        scene_vtile(a, lay, c, 16 * task, wcc);\n"
     "        __builtin_amdgcn_s_waitcnt(0xc07f);\n        G2K_TL(113 + 3 * task, fb == 0);\n"
     "        scene_vtile(a, lay, c, 16 * task, wcc);\n        __builtin_amdgcn_s_waitcnt(0xc07f);\n"
     "        G2K_TL(114 + 3 * task, fb == 0);\n      } else {\n"
     "        G2K_TL(118, fb == 0);\n        scene_kmats(c);\n        __builtin_amdgcn_s_waitcnt(0xc07f);\n"
     "        G2K_TL(119, fb == 0);\n        scene_kmats(c);\n        __builtin_amdgcn_s_waitcnt(0xc07f);\n"
     "        G2K_TL(120, fb == 0);"),
]
if os.environ.get("TL_WARM"):
    REPS += WARM
# TL_GRAD=1 (build): producer 0's first two gradient frames of chunk 0, four
# stamps each (after the M poll, after the first tile, before / after frame_grad)
GRADF = [
    ("  for (int fl = f0; fl < fend; fl += fstep) {\n    const int f = fb + fl;\n    const int ford",
     "  int g2k_gk = 0;\n  for (int fl = f0; fl < fend; fl += fstep) {\n    const int f = fb + fl;\n    const int ford"),
    ("    poll_flag(c.sMflag + fl, f + 1);                     // M of this frame (a producer's head)\n",
     "    poll_flag(c.sMflag + fl, f + 1);                     // M of this frame (a producer's head)\n"
     "    G2K_TL(71 + 4 * g2k_gk, slot == 0 && fb == 0 && t0 == 0 && g2k_gk < 2);\n"),
    ("                               c.sNllC, c.sNllA + slot * 12 * 64 + c.lane);\n",
     "                               c.sNllC, c.sNllA + slot * 12 * 64 + c.lane);\n"
     "      G2K_TL(72 + 4 * g2k_gk, slot == 0 && fb == 0 && t0 == 0 && g2k_gk < 2 && t == t0);\n"),
    ("    frame_grad(a, lay, c, fl, dm, slot);\n",
     "    G2K_TL(73 + 4 * g2k_gk, slot == 0 && fb == 0 && t0 == 0 && g2k_gk < 2);\n"
     "    frame_grad(a, lay, c, fl, dm, slot);\n"
     "    G2K_TL(74 + 4 * g2k_gk, slot == 0 && fb == 0 && t0 == 0 && g2k_gk < 2);\n    ++g2k_gk;\n"),
    ("      if (pw < R && grad_rec_tiles(ntact) < ntact) {    // the recurrence waves' frames' other tiles\n",
     "      G2K_TL(121, pw == 0 && fb == 0);\n"
     "      if (pw < R && grad_rec_tiles(ntact) < ntact) {    // the recurrence waves' frames' other tiles\n"),
]
if os.environ.get("TL_GRAD"):
    REPS += GRADF
# TL_VTILE=1 (build): producer 0's first V tile (window rows 0..15), four stamps
# (entry, after the k-loop's MFMAs, after the VG MFMAs, after the stores)
VTILE = [
    ("  const int nks = ((nact + 15) / 16) * 4;\n  f32x4 v0 =",
     "  G2K_TL(122, w0 == 0);\n  const int nks = ((nact + 15) / 16) * 4;\n  f32x4 v0 ="),
    ("  f32x4 vt;\n#pragma unroll\n  for (int i = 0; i < 4; ++i) vt[i] = v0[i] + v1[i];\n",
     "  f32x4 vt;\n#pragma unroll\n  for (int i = 0; i < 4; ++i) vt[i] = v0[i] + v1[i];\n"
     "  asm volatile(\"\" :: \"v\"(vt[0]), \"v\"(vt[3]));\n  G2K_TL(123, w0 == 0);\n"),
    ("  const int row = win ? r : lay.wcmax + (r - wcc);               // storage row\n",
     "  asm volatile(\"\" :: \"v\"(vg[0]), \"v\"(vg[3]));\n  G2K_TL(124, w0 == 0);\n"
     "  const int row = win ? r : lay.wcmax + (r - wcc);               // storage row\n"),
]
if os.environ.get("TL_VTILE"):
    REPS += VTILE
# TL_DWI=1 (build, train): producer 0's dWi tile run twice, stamped before /
# between / after (is the finalize's time the code's first fetch?)
DWI = [
    ("    if (n0 < c.nact) {\n      if (lay.fc >= F) dwi(c.sPos, lay.pp);\n      else dwi(a.pos + (size_t)c.s * a.d.W * Nmax * 2, 2 * Nmax);\n    }\n",
     "    G2K_TL(108, pw == 0 && t == 0);\n"
     "    if (n0 < c.nact) {\n      if (lay.fc >= F) dwi(c.sPos, lay.pp);\n      else dwi(a.pos + (size_t)c.s * a.d.W * Nmax * 2, 2 * Nmax);\n    }\n"
     "    asm volatile(\"\" :: \"v\"(acc4[0]));\n    G2K_TL(109, pw == 0 && t == 0);\n    acc4 = f32x4{0.f, 0.f, 0.f, 0.f};\n"
     "    if (n0 < c.nact) {\n      if (lay.fc >= F) dwi(c.sPos, lay.pp);\n      else dwi(a.pos + (size_t)c.s * a.d.W * Nmax * 2, 2 * Nmax);\n    }\n"
     "    asm volatile(\"\" :: \"v\"(acc4[0]));\n    G2K_TL(110, pw == 0 && t == 0);\n"),
]
if os.environ.get("TL_DWI"):
    REPS += DWI
FINE = {48: "heads loop entry", 49: "head 1", 50: "head 2", 51: "head 3", 52: "head 4", 53: "head 5", 54: "head 6", 55: "head 7+"}


def build():
    from multimodaltraj_2_amd import build as b
    from concurrent.futures import ThreadPoolExecutor
    src = os.environ.get("TL_SRC", os.path.join(ROOT, "multimodaltraj_2_amd", "csrc"))
    tmp = tempfile.mkdtemp(prefix="g2k_tl_")
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), tmp)
    p = os.path.join(tmp, "g2k_scene.hip")
    s = open(p).read()
    for a, r in REPS:
        assert s.count(a) == 1, a[:70]
        s = s.replace(a, r)
    open(p, "w").write(s + EXPORT)

    def comp(f):
        o = os.path.join(tmp, os.path.splitext(f)[0] + ".o")
        if f.endswith(".cpp"):
            cmd = [b.CXX, *b.CXX_FLAGS, "-c", "-o", o, os.path.join(tmp, f)]
        else:
            cmd = [b.HIPCC, *b.flags_for(f), "-c", "-o", o, os.path.join(tmp, f)]
        subprocess.run(cmd, check=True)
        return o

    files = sorted(f for f in os.listdir(tmp) if f.endswith((".hip", ".cpp")))
    with ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(comp, files))
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT, *objs], check=True)
    shutil.rmtree(tmp, ignore_errors=True)
    print(OUT)


def run(config, nstreams, split=0, cores=False):
    import torch
    from multimodaltraj_2_amd import _lib, frame_step as fs
    from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch
    lib = _lib.load(OUT)
    _lib._lib = lib
    for n in ("g2k_tl_copy", "g2k_tl_count"):
        getattr(lib, n).argtypes = [ctypes.c_void_p] + ([ctypes.c_int] if n == "g2k_tl_copy" else [])
    dev = torch.device("cuda", 0)
    cfg = dict(CONFIGS[config])
    if config in ("eth_ucy_loo_kfold4", "dense_crowd"):
        cfg["S"] //= 8
    S, Nmax, H = cfg["S"], cfg["Nmax"], cfg["H"]
    b = make_batch(S, Nmax, H, F=20, seed=1)
    base = b.to_device(dev)
    params = fs.init_params(Nmax, seed=0).to(dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
    K = min(3 * nstreams, 8192 // S)   # (the stamp buffer holds 8192 workgroups)
    plans = []
    for k in range(K):
        t = {key: (v.clone() if isinstance(v, torch.Tensor) else v) for key, v in base.items()}
        if os.environ.get("TL_TRAIN"):                  # train mode: the gradient launch
            from multimodaltraj_2_amd import train_step as ts
            plans.append(ts.TrainPlan(params, t["pos"], t["vislet"], t["G"], t["targets"],
                                      t["n_active"], t["h0"], n_frames=t["n_frames"],
                                      ped_mask=t["ped_mask"], stride=b.stride,
                                      stream=streams[k % nstreams], pred_layout="ped", split=split))
        else:
            plans.append(fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                                     t["h0"], n_frames=t["n_frames"], ped_mask=t["ped_mask"],
                                     stride=b.stride, stream=streams[k % nstreams], pred_layout="ped",
                                     split=split, coresident=cores))
    tags = {int(p.out.h.data_ptr() >> 8) & 0xffffffff: k for k, p in enumerate(plans)}
    for _ in range(3):
        for p in plans:
            p.run()
    torch.cuda.synchronize()
    lib.g2k_tl_reset()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(streams[0])
    for s in streams[1:]:
        s.wait_stream(streams[0])
    for p in plans:
        p.run()
    for s in streams[1:]:
        streams[0].wait_stream(s)
    e1.record(streams[0])
    torch.cuda.synchronize()
    wall_us = e0.elapsed_time(e1) * 1e3
    cnt = ctypes.c_uint(0)
    lib.g2k_tl_count(ctypes.byref(cnt))
    n = cnt.value
    assert n <= 8192, n
    buf = (ctypes.c_uint * (n * NREC))()
    assert lib.g2k_tl_copy(buf, n * NREC) == 0
    r = np.frombuffer(buf, dtype=np.uint32).reshape(n, NREC).astype(np.int64)
    # s_memtime counters are per XCD (not synchronised across XCDs): times
    # relative to the earliest start on the workgroup's own XCD
    xcc = r[:, 3] & 0xf
    t0 = np.zeros(n, dtype=np.int64)
    for x in np.unique(xcc):
        t0[xcc == x] = r[xcc == x, 4].min()
    rel = lambda col: (r[:, col] - t0) % (1 << 32)   # noqa: E731
    np_ = 4 if fs.step_coresidency(S, 20, H, Nmax, b.pos.shape[1], b.stride, cores) == 2 else 12
    if os.environ.get("TL_TRAIN"):
        np_ = 8
    start, ex = rel(4), np.max([rel(32 + w) for w in range(4 + np_)], axis=0)
    span_cyc = np.median([ex[xcc == x].max() for x in np.unique(xcc)])
    ghz = span_cyc / wall_us / 1e3
    print(f"{config} NP={np_} split={split} streams={nstreams} launches={K} "
          f"workgroups={n} wall {wall_us:.1f} us ({wall_us / K:.2f} per launch), clock ~{ghz:.2f} GHz")
    launch = np.array([tags.get(int(v), -1) for v in r[:, 1]])
    prod_end = np.max([rel(20 + p) for p in range(np_)], axis=0)
    heads = np.max([rel(8 + p) for p in range(np_)], axis=0)
    cols = dict(B2=rel(5), chain0=rel(6), chain_end=rel(7), heads=heads, prod_end=prod_end, exit=ex)
    for k in range(K):
        m = launch == k
        if not m.any():
            continue
        st = start[m]
        line = [f"launch {k:2d} (stream {k % nstreams}): wg {m.sum():3d} start {st.min() / ghz / 1e3:7.2f}-{st.max() / ghz / 1e3:7.2f} us"]
        for name, v in cols.items():
            d = (v[m] - st)
            line.append(f"{name} {np.median(d):6.0f}/{d.max():6.0f}")
        pe = np.array([rel(20 + p) for p in range(np_)])[:, m]
        pspread = pe.max(axis=0) - pe.min(axis=0)
        line.append(f"prod spread {np.median(pspread):6.0f}/{pspread.max():6.0f}")
        line.append(f"end {ex[m].max() / ghz / 1e3:7.2f} us")
        print("  ".join(line))
    # producer 0's heads: entry after B2 and each head's end (cycles, medians over all workgroups)
    e48 = rel(48) - rel(5)
    fine = [f"entry-B2 {np.median(e48):.0f}"]
    prev = rel(48)
    for k in range(49, 56):
        v = rel(k)
        ok = r[:, k] != 0
        if ok.sum() < n // 2:
            break
        fine.append(f"{FINE[k]} +{np.median((v - prev)[ok]):.0f}")
        prev = v
    print("producer 0:", "  ".join(fine))
    st = {"B1 rec0": rel(56) - start, "B1 prod0": rel(57) - start, "staged rec0": rel(58) - start,
          "staged prod0": rel(59) - start, "B2 rec0": rel(5) - start, "chain0": rel(6) - start}
    if np_ == 4:
        print("staging task done per producer (medians):", "  ".join(f"p{p} {np.median(rel(24 + p) - start):.0f}" for p in range(4)))
    nw = 4 + np_
    print("B1 arrival per wave (medians):", "  ".join(f"w{w} {np.median(rel(96 + w) - start):.0f}" for w in range(nw)))
    print("B2 arrival per wave (medians):", "  ".join(f"w{w} {np.median(rel(80 + w) - start):.0f}" for w in range(nw)))
    if np.any(r[:, 113] != 0):
        d = lambda i, j: np.median(((r[:, j] - r[:, i]) % (1 << 32))[r[:, j] != 0])   # noqa: E731
        print(f"warm test: vtile0 first {d(112, 113):.0f} second {d(113, 114):.0f}; "
              f"vtile1 first {d(115, 116):.0f} second {d(116, 117):.0f}; "
              f"kmats first {d(118, 119):.0f} second {d(119, 120):.0f}")
    if np.any(r[:, 124] != 0):
        d = lambda i, j: np.median(((r[:, j] - r[:, i]) % (1 << 32))[(r[:, j] != 0) & (r[:, i] != 0)])   # noqa: E731
        print(f"vtile 0: entry at {np.median((rel(122) - start)[r[:, 122] != 0]):.0f}, k-loop {d(122, 123):.0f}, "
              f"VG {d(123, 124):.0f}, to staged {d(124, 59):.0f}")
    if np.any(r[:, 110] != 0):
        d = lambda i, j: np.median(((r[:, j] - r[:, i]) % (1 << 32))[(r[:, j] != 0) & (r[:, i] != 0)])   # noqa: E731
        print(f"dWi tile (producer 0): first run {d(108, 109):.0f}, second run {d(109, 110):.0f}")
    print("lead (cycles after start, medians):", "  ".join(f"{k} {np.median(v):.0f}" for k, v in st.items()))
    pro = {"start - entry": (r[:, 4] - r[:, 70]) % (1 << 32), "pos dma issued": rel(60) - start, "segments issued": rel(61) - start,
           "rec0 scalars": rel(62) - start, "loads landed (w0 or p0)": rel(63) - start}
    if os.environ.get("TL_TRAIN"):
        tr = {"heads done": rel(8) - start, "grad frames done": rel(44) - start, "chunk synced": rel(45) - start,
              "tickets (all metrics)": rel(46) - start, "dWi done": rel(47) - start,
              "prod0 end": rel(20) - start, "chain end": rel(7) - start, "exit": ex - start,
              "flushed": rel(64) - start, "metrics published": rel(65) - start,
              "priv summed": rel(66) - start, "rec0 grad frame done": rel(67) - start}
        if np.any(r[:, 74] != 0):
            d = lambda i, j: np.median(((r[:, j] - r[:, i]) % (1 << 32))[(r[:, j] != 0) & (r[:, i] != 0)])   # noqa: E731
            ntl = (np.asarray(b.n_active)[(r[:, 0] - 1) % S] + 15) // 16
            for nt in np.unique(ntl):
                m = ntl == nt
                dm_ = lambda i, j: np.median(((r[:, j] - r[:, i]) % (1 << 32))[m & (r[:, j] != 0) & (r[:, i] != 0)])   # noqa: E731
                for g in range(2):
                    o = 71 + 4 * g
                    print(f"  {nt}-tile scenes, producer 0 gradient frame {g}: M ready at {np.median((rel(o) - start)[m]):.0f}, "
                          f"first tile {dm_(o, o + 1):.0f}, other tiles {dm_(o + 1, o + 2):.0f}, frame_grad {dm_(o + 2, o + 3):.0f}"
                          + (f", to next frame {dm_(o + 3, o + 4):.0f}" if g == 0 else ""))
                if np.any(r[m, 121] != 0):
                    print(f"  {nt}-tile scenes, producer 0: own frames done at {np.median((rel(121) - start)[m]):.0f}, "
                          f"with the recurrence frames' other tiles at {np.median((rel(44) - start)[m]):.0f}")
        print("train, producer 0 (cycles after start, medians):", "  ".join(f"{k} {np.median(v):.0f}" for k, v in tr.items()))
        ntile = (np.asarray(b.n_active)[(r[:, 0] - 1) % S] + 15) // 16
        for nt in np.unique(ntile):
            m = ntile == nt
            print(f"  scenes with {nt} tile(s) ({m.sum()} wg):", "  ".join(f"{k} {np.median(v[m]):.0f}" for k, v in tr.items()),
                  f" exit max {(ex - start)[m].max():.0f}")
    print("prologue (cycles after start, medians):", "  ".join(f"{k} {np.median(v):.0f}" for k, v in pro.items()))
    # per XCD: medians / maxima of B1, B2 and the exit (the launch ends with its slowest workgroup)
    b1 = rel(56) - start
    print("per XCD (B1 med/max, B2 med/max, exit med/max):", "  ".join(
        f"x{int(x)} {np.median(b1[xcc == x]):.0f}/{b1[xcc == x].max():.0f} "
        f"{np.median((rel(5) - start)[xcc == x]):.0f}/{(rel(5) - start)[xcc == x].max():.0f} "
        f"{np.median((ex - start)[xcc == x]):.0f}/{(ex - start)[xcc == x].max():.0f}" for x in np.unique(xcc)))
    # co-residency: workgroups sharing a CU (XCC_ID, HW_ID[15:8]) at the same time
    cu = (r[:, 3] << 8) | ((r[:, 2] >> 8) & 0xff)
    over = np.zeros(n, dtype=int)
    order = np.argsort(cu)
    for key in np.unique(cu):
        idx = np.nonzero(cu == key)[0]
        for i in idx:
            over[i] = int(((start[idx] < ex[i]) & (ex[idx] > start[i])).sum()) - 1
    print("distinct CUs", len(np.unique(cu)), "; workgroups overlapping another on their CU:",
          {int(v): int((over == v).sum()) for v in np.unique(over)})


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    else:
        run(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1,
            int(sys.argv[3]) if len(sys.argv) > 3 else 0, len(sys.argv) > 4 and sys.argv[4] == "on")
