"""A/B timing of source variants of the scene kernel (development tool, not
product code).  Each variant is a set of text replacements applied to a temp
copy of multimodaltraj_2_amd/csrc; the copy is built into /tmp and timed on
the bench workload (HIP events, reference-mode step and train step).

usage: python tools/ab_time.py --build VARIANT ...       (CPU host: into tools/ab/)
       python tools/ab_time.py [CONFIG] [VARIANT ...]   (GPU: timelines / times)
       python tools/ab_time.py --rounds K [CONFIG] VARIANT ...   (interleaved A/B)"""
import ctypes
import os
import shutil
import subprocess
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multimodaltraj_2_amd import _lib, build, frame_step as fs, train_step as ts  # noqa: E402
from multimodaltraj_2_amd.synthetic import CONFIGS, make_batch  # noqa: E402

SCENE = "g2k_scene.hip"
# diagnostic build: s_memtime stamps (low 32 bits) of scene 0's producer 0 /
# recurrence wave 0 written past the gradient rows of a widened workspace
STAMP_DEF = """
__device__ unsigned g2k_stamp_buf[4096 * 64];
#define G2K_ST(k, cond) do { if ((cond) && c.lane == 0) { \\
  const unsigned long long _t = __builtin_amdgcn_s_memtime(); \\
  g2k_stamp_buf[(size_t)c.s * 64 + (k)] = (unsigned)_t; } } while (0)
"""
STAMP_EXPORT = """
extern "C" int g2k_stamp_copy(unsigned* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g2k::g2k_stamp_buf), (size_t)n * 4, 0,
                                  hipMemcpyDeviceToHost);
}
"""
P0 = "c.wv == kRecW"
STAMPS = [
    ("namespace g2k {\nnamespace {\n\nconstexpr int kSceneChunk", "namespace g2k {\n" + STAMP_DEF + "namespace {\n\nconstexpr int kSceneChunk"),
    ("int scene_step_launch(const StepArgs& a, hipStream_t st) {", "int scene_step_launch(const StepArgs& a, hipStream_t st) {\n  (void)0;"),
    ("  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;",
     "  G2K_ST(0, c.tid == 0);\n  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;"),
    ("    scene_stage<64 * (kRecW + NP), NP, 0>(a, lay, c, fb, cnt, false, [] {});",
     "    scene_stage<64 * (kRecW + NP), NP, 0>(a, lay, c, fb, cnt, false, [] {});\n    G2K_ST(1, " + P0 + " && fb == 0);"),
    ("    // phase 2 — predictions and errors (GRAD: and the gradient)",
     "    G2K_ST(2, " + P0 + " && fb == 0);\n    // phase 2 — predictions and errors (GRAD: and the gradient)"),
    ("        frame_grad(a, lay, c, pw + fi * NP, dm);",
     "        G2K_ST(3 + fi, " + P0 + " && fb == 0 && fi < 5);\n        frame_grad(a, lay, c, pw + fi * NP, dm);\n        G2K_ST(8 + fi, " + P0 + " && fb == 0 && fi < 4);"),
    ("      poll_word(c.sGseq, NP * (fb / lay.fc + 1));",
     "      G2K_ST(24 + pw, fb == 0);\n      poll_word(c.sGseq, NP * (fb / lay.fc + 1));\n      G2K_ST(12, " + P0 + " && fb == 0);"),
    ("      if (ntact > 0) grad_chunk_flush(a, lay, c, fb, cnt, NP);   // (no active pedestrian: all zero)",
     "      if (ntact > 0) grad_chunk_flush(a, lay, c, fb, cnt, NP);   // (no active pedestrian: all zero)\n      G2K_ST(13, " + P0 + " && fb == 0);"),
    ("  ticket = __builtin_amdgcn_readfirstlane(ticket);", "  ticket = __builtin_amdgcn_readfirstlane(ticket);\n  G2K_ST(14, " + P0 + ");"),
    ("  poll_word(c.sTicket, NP);", "  poll_word(c.sTicket, NP);\n  G2K_ST(15, " + P0 + ");"),
    ("  poll_word(c.sGseq + 1, NP);", "  poll_word(c.sGseq + 1, NP);\n  G2K_ST(11, " + P0 + ");"),
    ("  // the small blocks and dWo, entry by entry", "  G2K_ST(16, " + P0 + ");\n  // the small blocks and dWo, entry by entry"),
    ("  rc.store(a.h_out", "  G2K_ST(20, c.wv == 0);\n  rc.store(a.h_out"),
    ("    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first",
     "    G2K_ST(21, " + P0 + ");\n    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first\n    G2K_ST(22, " + P0 + ");"),
    ("    if (c.tid < lay.fc) {                                // flags hold (global frame + 1)",
     "    G2K_ST(23, " + P0 + ");\n    if (c.tid < lay.fc) {                                // flags hold (global frame + 1)"),
    ("  c.ntact = (c.nact + 15) >> 4;                        // tiles holding active pedestrians",
     "  c.ntact = (c.nact + 15) >> 4;                        // tiles holding active pedestrians\n  G2K_ST(25, " + P0 + ");"),
    ("    scene_producer<NP, GRAD>(a, lay, c);", "  { G2K_ST(17, " + P0 + "); scene_producer<NP, GRAD>(a, lay, c); }"),
    ("  __syncthreads();                                              // B1: window + weights landed",
     "  G2K_ST(18, " + P0 + " && fb == 0);\n  __syncthreads();\n  G2K_ST(19, " + P0 + " && fb == 0);"),
    ("      const FrameHeadOut hd =", "      G2K_ST(30 + 3 * (fl / NP), " + P0 + " && fb == 0 && fl < 3 * NP);\n      const FrameHeadOut hd ="),
    ("      if (L < kL && q < 2) {\n        float* m = c.sMring", "      G2K_ST(31 + 3 * (fl / NP), " + P0 + " && fb == 0 && fl < 3 * NP);\n      if (L < kL && q < 2) {\n        float* m = c.sMring"),
    ("        lds_store_flag(c.sFlag + fl, f + 1);\n      }\n", "        lds_store_flag(c.sFlag + fl, f + 1);\n      }\n      G2K_ST(32 + 3 * (fl / NP), " + P0 + " && fb == 0 && fl < 3 * NP);\n"),
]
TILE = [
    ("f32x4 (&dm)[2], f32x4& dWoT, AfterTargets after_targets) {", "f32x4 (&dm)[2], f32x4& dWoT, AfterTargets after_targets, const StepArgs& a, const SceneCtx& c) {\n  G2K_ST(40, " + P0 + " && t == 0);"),
    ("c.nact, t, L, q, acc, lsum, dm, dWoT, after_targets);", "c.nact, t, L, q, acc, lsum, dm, dWoT, after_targets, a, c);"),
    ("  after_targets();\n", "  G2K_ST(41, " + P0 + " && t == 0);\n  after_targets();\n"),
    ("  // errors: d = Y - target", "  G2K_ST(42, " + P0 + " && t == 0);\n  // errors: d = Y - target"),
    ("    // dY into the scratch [r][n]", "    G2K_ST(43, " + P0 + " && t == 0);\n    // dY into the scratch [r][n]"),
    ("    wave_lds_sync();\n    // dm += dY", "    G2K_ST(44, " + P0 + " && t == 0);\n    wave_lds_sync();\n    // dm += dY"),
    ("    wave_lds_sync();                       // scratch reads done", "    G2K_ST(45, " + P0 + " && t == 0);\n    wave_lds_sync();                       // scratch reads done"),
    ("      poll_flag(c.sMflag + fl, f + 1);         // M of this frame", "      G2K_ST(46, " + P0 + " && t == 0);\n      poll_flag(c.sMflag + fl, f + 1);         // M of this frame"),
    ("        if (lay.dwo_seq) {\n          asm volatile", "        G2K_ST(47, " + P0 + " && t == 0);\n        if (lay.dwo_seq) {\n          asm volatile"),
]
# forward timeline: scene's producer 0 (P0) and recurrence wave 0 (R0);
# slot 27 / 28: s_memrealtime (100 MHz) at start / end of R0 (dispatch skew)
R0 = "c.wv == 0"
TL_FWD = [
    ("namespace g2k {\nnamespace {\n\nconstexpr int kSceneChunk", "namespace g2k {\n" + STAMP_DEF + "namespace {\n\nconstexpr int kSceneChunk"),
    ("  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;",
     "  G2K_ST(0, c.tid == 0);\n  if (c.wv == 0 && c.lane == 0) g2k_stamp_buf[(size_t)c.s * 64 + 27] = (unsigned)__builtin_amdgcn_s_memrealtime();\n"
     "  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;"),
    ("    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first",
     "    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first\n    G2K_ST(1, " + P0 + ");"),
    ("    c.ntact = (c.nact + 15) >> 4;                      // tiles holding active pedestrians",
     "    c.ntact = (c.nact + 15) >> 4;                      // tiles holding active pedestrians\n    G2K_ST(3, " + P0 + ");"),
    ("  __builtin_amdgcn_s_barrier();                                 // B1: window + weights landed",
     "  G2K_ST(4, " + P0 + " && fb == 0);\n  __builtin_amdgcn_s_barrier();\n  G2K_ST(5, " + P0 + " && fb == 0);"),
    ("  __builtin_amdgcn_s_barrier();                                 // B2: V, VG, K1, K2",
     "  G2K_ST(51, " + P0 + " && fb == 0);\n  __builtin_amdgcn_s_barrier();\n  G2K_ST(6, " + P0 + " && fb == 0);"),
    ("      const FrameHeadOut hd =", "      G2K_ST(7 + 2 * (i / NP), " + P0 + " && fb == 0 && i < 3 * NP);\n      const FrameHeadOut hd ="),
    ("        if (lane == 0) lds_store_flag(c.sMflag + fl, f + 1);\n      }\n",
     "        if (lane == 0) lds_store_flag(c.sMflag + fl, f + 1);\n      }\n      G2K_ST(8 + 2 * (i / NP), " + P0 + " && fb == 0 && i < 3 * NP);\n"),
    ("        poll_flag(c.sMflag + fl, f + 1);         // M of this frame (maybe another producer's)",
     "        G2K_ST(13 + 2 * k, " + P0 + " && k < 6);\n        poll_flag(c.sMflag + fl, f + 1);         // M of this frame (maybe another producer's)\n        G2K_ST(14 + 2 * k, " + P0 + " && k < 6);"),
    ("  publish_metrics(a, c, pw, GRAD ? NP + kRecW : NP, acc, lsum, GRAD);",
     "  G2K_ST(25, " + P0 + ");\n  publish_metrics(a, c, pw, GRAD ? NP + kRecW : NP, acc, lsum, GRAD);\n  G2K_ST(50, " + P0 + ");"),
    ("        rc.step_seq(b, z, c.sRed + ((g + 1) & 1) * kRB, seq, g + 3, c.wv, c.q, c.L, c.sFlag + fn,\n                    as_lane + fn * kD * kD, fln, bn, g + 1 == c.nf);",
     "        rc.step_seq(b, z, c.sRed + ((g + 1) & 1) * kRB, seq, g + 3, c.wv, c.q, c.L, c.sFlag + fn,\n                    as_lane + fn * kD * kD, fln, bn, g + 1 == c.nf);\n        G2K_ST(30 + g, " + R0 + " && g < 20);"),
    ("  rc.store(a.h_out + (size_t)c.s * kD * H, H, c.wv, c.q, c.L,\n           c.nf > 0 ? c.sRed + (c.nf & 1) * kRB : nullptr);",
     "  rc.store(a.h_out + (size_t)c.s * kD * H, H, c.wv, c.q, c.L,\n           c.nf > 0 ? c.sRed + (c.nf & 1) * kRB : nullptr);\n  G2K_ST(26, " + R0 + ");\n"
     "  if (c.wv == 0 && c.lane == 0) g2k_stamp_buf[(size_t)c.s * 64 + 28] = (unsigned)__builtin_amdgcn_s_memrealtime();"),
    ("      if (c.lane == 0) lds_store_flag(seq + c.wv, 2);\n    });",
     "      if (c.lane == 0) lds_store_flag(seq + c.wv, 2);\n    });\n  G2K_ST(52, " + R0 + ");"),
]


# one frame of the recurrence in detail (g = 17, 18): R0 before / after its
# poll, every wave's publish
TL_REC = TL_FWD + [
    ("        poll_red(seq + (c.L & 3), g + 2, c.sRed + (g & 1) * kRB + (c.L & 3) * 16 + 4 * c.q, z);",
     "        G2K_ST(53, " + R0 + " && g == 17);\n"
     "        poll_red(seq + (c.L & 3), g + 2, c.sRed + (g & 1) * kRB + (c.L & 3) * 16 + 4 * c.q, z);\n"
     "        G2K_ST(54, " + R0 + " && g == 17);\n        G2K_ST(59, " + R0 + " && g == 18);"),
    ("        G2K_ST(30 + g, " + R0 + " && g < 20);",
     "        G2K_ST(30 + g, " + R0 + " && g < 20);\n        G2K_ST(55 + c.wv, c.wv > 0 && g == 17);"),
]


# the same stamps kept in LDS (no global store, so no vmcnt wait behind a
# stamp) and copied out after a final barrier
LDS_STAMP_DEF = """
__device__ unsigned g2k_stamp_buf[4096 * 160];
__shared__ unsigned g2k_lds_stamp[160];
#define G2K_ST(k, cond) do { if ((cond) && (threadIdx.x & 63) == 0) { \\
  g2k_lds_stamp[(k)] = (unsigned)__builtin_amdgcn_s_memtime(); } } while (0)
"""
HEAD_ST = "wrow0 == 0"


def lds_stamps(reps, head=True):
    out = []
    for a, b in reps:
        b = b.replace(STAMP_DEF, LDS_STAMP_DEF)
        b = b.replace("g2k_stamp_buf[(size_t)c.s * 64 + 27]", "g2k_lds_stamp[27]")
        b = b.replace("g2k_stamp_buf[(size_t)c.s * 64 + 28]", "g2k_lds_stamp[28]")
        out.append((a, b))
    out += [
        ('  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup',
         '  __syncthreads();\n  if (c.tid < 160) g2k_stamp_buf[(size_t)c.s * 160 + c.tid] = g2k_lds_stamp[c.tid];\n'
         '  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup'),
    ]
    if head:
        out += [
        ("    f32x4 eN = {0.f, 0.f, 0.f, 0.f};\n#pragma unroll\n    for (int ks = 0; ks < 3; ++ks) eN = mfma4(ka[ks], ua[ks], eN);",
         "    G2K_ST(60, " + HEAD_ST + ");\n    f32x4 eN = {0.f, 0.f, 0.f, 0.f};\n#pragma unroll\n    for (int ks = 0; ks < 3; ++ks) eN = mfma4(ka[ks], ua[ks], eN);"),
        ("    __builtin_amdgcn_sched_barrier(0);\n    attn_weights(aA, as_dst, L, q);",
         "    G2K_ST(61, " + HEAD_ST + " && aA[0] != 12345.f);\n    __builtin_amdgcn_sched_barrier(0);\n    attn_weights(aA, as_dst, L, q);"),
        ("  if ((threadIdx.x & 63) == 0) lds_store_flag(as_flag, flag_val);",
         "  if ((threadIdx.x & 63) == 0) lds_store_flag(as_flag, flag_val);\n  G2K_ST(62, " + HEAD_ST + ");"),
    ]
    return out


# I-cache test: the recurrence waves' first head executed twice by the same
# code (a loop, not unrolled), stamped before / between / after (R0)
TL_ICACHE = [
    ("    const int fl = c.wv;\n    const bool mine = c.X == 1 || fl % c.X == 0;\n    frame_head(",
     "    const int fl = c.wv;\n    const bool mine = c.X == 1 || fl % c.X == 0;\n"
     "    G2K_ST(76, " + R0 + ");\n"
     "#pragma unroll 1\n    for (int rep = 0; rep < 2; ++rep) {\n    frame_head("),
    ("               nullptr, c.L, c.q, /*want_m=*/false);\n    __builtin_amdgcn_s_setprio(0);\n  }\n",
     "               nullptr, c.L, c.q, /*want_m=*/false);\n    G2K_ST(77 + rep, " + R0 + ");\n    }\n    __builtin_amdgcn_s_setprio(0);\n  }\n"),
]


# the producers' lead-in between the staging barrier and the first head
TL_GAP = [
    ("    if (fb == 0) act_bits = scene_act_bits(c, scene_mask_word(a, lay, c));   // (the row is in LDS)",
     "    G2K_ST(70, " + P0 + " && fb == 0);\n    if (fb == 0) act_bits = scene_act_bits(c, scene_mask_word(a, lay, c));   // (the row is in LDS)\n    G2K_ST(71, " + P0 + " && fb == 0);"),
    ("    float rm[4];\n    scene_rm(lay, c, rm);\n    // phase 1",
     "    G2K_ST(72, " + P0 + " && fb == 0);\n    float rm[4];\n    scene_rm(lay, c, rm);\n    // phase 1"),
    ("               nullptr, c.L, c.q, /*want_m=*/false);\n    __builtin_amdgcn_s_setprio(0);\n  }\n",
     "               nullptr, c.L, c.q, /*want_m=*/false);\n    __builtin_amdgcn_s_setprio(0);\n  }\n  G2K_ST(74, " + R0 + ");\n"),
    ("    if (live) {\n      __builtin_amdgcn_s_setprio(2);",
     "    G2K_ST(75, " + R0 + " && fb == 0);\n    if (live) {\n      __builtin_amdgcn_s_setprio(2);"),
]


# I-cache experiment: every producer runs the staging and frame-head code once
# on whatever LDS holds while the prologue's DMA is in flight
WARM = [
    ("  if (VMC > 0 && fb == 0 && hl) asm volatile(\"s_waitcnt vmcnt(%0)\" ::\"n\"(VMC) : \"memory\");",
     "  if (fb == 0 && c.wv >= kRecW) {\n"
     "    scene_vtile(a, lay, c, 0, wcc);\n    scene_kmats(c);\n    float rm0[4] = {0.f, 0.f, 0.f, 0.f};\n"
     "    (void)frame_head(c.sm, c.sV, c.sVG, 0, lay.wcmax, rm0, a.lambda, c.sRing + (c.wv - kRecW) * kD * kD, reinterpret_cast<int*>(c.sm + SM_SPARE), 0,\n"
     "                     nullptr, nullptr, nullptr, c.L, c.q);\n  }\n"
     "  if (VMC > 0 && fb == 0 && hl) asm volatile(\"s_waitcnt vmcnt(%0)\" ::\"n\"(VMC) : \"memory\");"),
]


# inside the forward tile (P0's LAST tile survives): entry, Y done, targets
# consumed, stores issued, error terms done
PT = "!GRAD && __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 4"
TL_TILE = [
    ("  const int n0 = 16 * t, n = n0 + L;\n  const bool hi = q < 2;",
     "  G2K_ST(40, " + PT + ");\n  const int n0 = 16 * t, n = n0 + L;\n  const bool hi = q < 2;"),
    ("  // errors: d = Y - target, (x, y) pairs in registers (v = 0, 1 and 2, 3)",
     "  G2K_ST(41, " + PT + " && y0[0] != 12345.f && y1[0] != 12345.f);\n  // errors: d = Y - target, (x, y) pairs in registers (v = 0, 1 and 2, 3)"),
    ("  after_targets();\n  asm volatile(\"\" ::: \"memory\");                           // ... then the stores",
     "  G2K_ST(42, " + PT + " && d0[0] != 12345.f && d1[3] != 12345.f);\n  after_targets();\n  asm volatile(\"\" ::: \"memory\");                           // ... then the stores"),
    ("  float ea = 0.f, eb = 0.f, ec = 0.f, el2 = 0.f;",
     "  G2K_ST(43, " + PT + ");\n  float ea = 0.f, eb = 0.f, ec = 0.f, el2 = 0.f;"),
    ("  if (GRAD) {\n#pragma unroll\n    for (int v = 0; v < 4; ++v) {\n      d0[v] = has_t ? d0[v] : 0.f;",
     "  G2K_ST(44, " + PT + " && acc[0] != 12345.f);\n  if (GRAD) {\n#pragma unroll\n    for (int v = 0; v < 4; ++v) {\n      d0[v] = has_t ? d0[v] : 0.f;"),
]


# every wave's own DMA wait before B1 (wave w -> slot 39 + w, w >= 1)
TL_B1 = [

    ("    c.ntact = (c.nact + 15) >> 4;                      // tiles holding active pedestrians",
     "    c.ntact = (c.nact + 15) >> 4;                      // tiles holding active pedestrians\n    G2K_ST(112 + c.wv, true);"),
    ("  // every kernel-argument line the prologue reads, in ONE scalar-load round",
     "  G2K_ST(80 + (threadIdx.x >> 6), true);\n  // every kernel-argument line the prologue reads, in ONE scalar-load round"),
    ("    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first",
     "    G2K_ST(96 + c.wv, true);\n    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first"),
    ("  __builtin_amdgcn_s_waitcnt(0x0070);                           // vmcnt(0) lgkmcnt(0)",
     "  G2K_ST(128 + c.wv, fb == 0);\n  __builtin_amdgcn_s_waitcnt(0x0070);                           // vmcnt(0) lgkmcnt(0)"),
    ("  __builtin_amdgcn_s_barrier();                                 // B1: window + weights landed",
     "  G2K_ST(64 + c.wv, fb == 0);\n  __builtin_amdgcn_s_barrier();                                 // B1: window + weights landed"),


]


# position window by 1-KiB LDS-DMA instructions into unpadded rows
POS1K = [
    ("  s.pp = 2 * Nmax + 4;", "  s.pp = 2 * Nmax;"),
    ("    if (wide) {\n      for (int i = 0; i < Nmax / 2; i += 64)\n        if (i + c.lane < Nmax / 2) dma16(g + 4 * (i + c.lane), d + 4 * i);\n    } else {",
     "    if (wide) {\n      if (r == c.wv) dma_copy_n<NT>(src, c.sPos, wcc * Nmax / 2, c.wv, c.lane);\n    } else {"),
]


# minimal stamps: every wave's exit (slot 64 + wave), R0's start (0)
TL_END = [
    ("namespace g2k {\nnamespace {\n\nconstexpr int kSceneChunk", "namespace g2k {\n" + STAMP_DEF + "namespace {\n\nconstexpr int kSceneChunk"),
    ("  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;",
     "  G2K_ST(0, c.tid == 0);\n  if (c.tid == 0) g2k_stamp_buf[(size_t)c.s * 64 + 27] = (unsigned)__builtin_amdgcn_s_memrealtime();\n"
     "  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;"),
    ('  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup',
     '  G2K_ST(64 + c.wv, true);\n  if (c.lane == 0) g2k_stamp_buf[(size_t)c.s * 64 + 28] = (unsigned)__builtin_amdgcn_s_memrealtime();\n'
     '  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup'),
]


def tl_end_print(st, t):
    import numpy as np
    rt = st[:, 27:29].copy()
    rel = (st - st[:, :1]) % (1 << 32)
    rel[:, 27:29] = 0
    span = (rt[:, 1] - rt[:, 0]) % (1 << 32)         # 100 MHz ticks, wave 0 start -> a late wave's exit
    cyc = rel[:, 64:80].max(1)
    ok = span > 0
    if ok.any():
        print("in-kernel clock (cycles / realtime, median over WGs): %.3f GHz; WG start spread %d ticks, "
              "last WG end - first WG start %d ticks" % (float(np.median(cyc[ok] / (span[ok] * 10.0))),
                                                      int(rt[:, 0].max() - rt[:, 0].min()),
                                                      int(rt[:, 1].max() - rt[:, 0].min())))
    print("WG duration (wave 0 start -> last wave exit, cycles): median", int(np.median(rel[:, 64:80].max(1))),
          "max", int(rel[:, 64:80].max()))
    ends = rel[:, 64:80]
    na = t["n_active"].cpu().numpy()
    print("wave exits (median over scenes, waves 0..15):", [int(x) for x in np.median(ends, axis=0)])
    for lo, hi in ((0, 8), (8, 16), (16, 24), (24, 33)):
        m = (na >= lo) & (na < hi)
        if m.any():
            e = ends[m]
            print(f"  n_active in [{lo},{hi}): {int(m.sum())} scenes; recurrence exit {int(np.median(e[:, :4].max(1)))}, "
                  f"producers exit {int(np.median(e[:, 4:].max(1)))}, max over these scenes: rec {int(e[:, :4].max())} prod {int(e[:, 4:].max())}")


def tl_rec_print(st, t):
    import numpy as np
    tl_fwd_print(st, t)
    rel = (st - st[:, :1]) % (1 << 32)
    med = np.median(rel, axis=0)
    print("frame 17 (median): R0 poll start", int(med[53]), "poll end", int(med[54]), "R0 published",
          int(med[47]), "waves 1-3 published", [int(med[56 + w]) for w in range(3)],
          "R0 frame 18 poll end", int(med[59]))


def tl_fwd_print(st, t):
    import numpy as np
    S = st.shape[0]
    rs = st[:, 27]
    re = st[:, 28]
    t0 = rs.min()
    print("realtime (10 ns ticks) start spread: min 0 max", int(rs.max() - t0),
          " end: min", int(re.min() - t0), "max", int(re.max() - t0),
          " median duration", float(np.median(re - rs)))
    names = {1: "dma issued", 3: "nact", 4: "B1 wait", 5: "B1", 51: "stage done", 6: "B2",
             7: "h0s", 8: "h0e", 9: "h1s", 10: "h1e", 11: "h2s", 12: "h2e", 25: "prod done",
             50: "published", 52: "R0 at stage", 26: "recur stored"}
    for sc in (0, S // 2, S - 1):
        r = st[sc]
        rel = (r - r[0]) % (1 << 32)
        print(f"scene {sc} n_active {int(t['n_active'][sc])}: " +
              "  ".join(f"{v}:{rel[k]}" for k, v in names.items()))
        print("   items (poll start, poll end):", " ".join(f"({rel[13 + 2 * k]},{rel[14 + 2 * k]})" for k in range(6)))
        print("   recurrence frame ends:", " ".join(str(rel[30 + g]) for g in range(20)))
    # the scenes that end last (realtime), with their two roles' ends
    rel = (st - st[:, :1]) % (1 << 32)
    last = np.argsort(re)[-6:]
    print("latest-ending scenes (scene, n_active, end tick, R0 stored, P0 published):",
          [(int(k), int(t["n_active"][k]), int(re[k] - t0), int(rel[k][26]), int(rel[k][50])) for k in last])
    print("end tick by n_active (mean):", {int(n): round(float((re - t0)[t["n_active"].cpu().numpy() == n].mean()), 1)
                                          for n in sorted(set(t["n_active"].cpu().numpy().tolist()))[::4]})
    med = np.median(rel, axis=0)
    print("median:", "  ".join(f"{v}:{int(med[k])}" for k, v in names.items()))
    print("median recurrence frame ends:", " ".join(str(int(med[30 + g])) for g in range(20)))
    print("median items:", " ".join(f"({int(med[13 + 2 * k])},{int(med[14 + 2 * k])})" for k in range(6)))


NO_RECUR = [("  const bool live = a.h_in != nullptr && c.x == 0;   // (the scene's first workgroup)",
             "  const bool live = false;")]
NO_TILES = [("    const int nitems = own.n * ntact > pw ? (own.n * ntact - pw + NP - 1) / NP : 0;   // forward",
             "    const int nitems = 0;")]
NO_RECUR_SCENE = {SCENE: NO_RECUR}
# the producers' heads before the tile set-up (mask bits, item counts, the
# first targets' loads)
_SETUP = """    if (fb == 0) act_bits = scene_act_bits(c, scene_mask_word(a, lay, c));   // (the row is in LDS)
    const OwnFrames own = own_frames(fb, cnt, c.X, c.x);
    ofo = own.fo;
    const int nitems = own.n * ntact > pw ? (own.n * ntact - pw + NP - 1) / NP : 0;   // forward
    // GRAD: this producer's own frames (ordinals) pw, pw + NP, ... < gend of
    // the chunk (the last R own frames of the last chunk go to the
    // recurrence waves)
    const int R = GRAD && fb + lay.fc >= c.nf ? grad_rec_frames(own.n, NP) : 0;
    const int gend = own.n - R;
    // the first tiles' targets: in flight during the heads (GRAD: one buffer
    // and the balancing stores, see grad_frames)
    if (GRAD) {
      load_targets(tgr, Nmax, c.nact, fb, own.fo + c.X * pw, 0, pw < gend, L, q, tgA, lay.tfb);
      balance_stores<PM>(a);
    } else {
      load_item(fb, nitems, 0, tgA);
      load_item(fb, nitems, 1, tgB);
    }
"""
_SETUP_AFTER = _SETUP.replace("""    if (fb == 0) act_bits = scene_act_bits(c, scene_mask_word(a, lay, c));   // (the row is in LDS)
    const OwnFrames own = own_frames(fb, cnt, c.X, c.x);
    ofo = own.fo;
""", """    if (fb == 0) act_bits = scene_act_bits(c, scene_mask_word(a, lay, c));   // (the row is in LDS)
    ofo = own.fo;
""")
HEADS_FIRST = [
    (_SETUP, "    const OwnFrames own = own_frames(fb, cnt, c.X, c.x);\n"),
    ("    // phase 2 — predictions and errors (GRAD: and the gradient)\n",
     _SETUP_AFTER + "    // phase 2 — predictions and errors (GRAD: and the gradient)\n"),
]
# every producer's first head ahead of the chunk loop (and its set-up)
PEEL = [
    ("  for (int fb = 0; fb < c.nf; fb += lay.fc) {\n    const int cnt = (c.nf - fb) < lay.fc ? (c.nf - fb) : lay.fc;\n    if (fb > 0) {\n      scene_pos_dma<64 * (kRecW + NP)>",
     "  int peeled = 0;\n"
     "  if (c.nf > 0) {\n"
     "    const int cnt = c.nf < lay.fc ? c.nf : lay.fc;\n"
     "    const OwnFrames own = own_frames(0, cnt, c.X, c.x);\n"
     "    const bool all_heads = a.h_in != nullptr && c.x == 0;\n"
     "    const int nrh = all_heads ? rec_head_frames(lay, c) : 0;\n"
     "    if (pw < (all_heads ? cnt : own.n)) {\n"
     "      peeled = NP;\n"
     "      const int fl = all_heads ? pw : own.fo + c.X * pw;\n"
     "      const int f = fl;\n"
     "      const bool mine = !all_heads || c.X == 1 || f % c.X == c.x;\n"
     "      if (!(fl < nrh && !mine)) {\n"
     "        float rm[4];\n"
     "        scene_rm(lay, c, rm);\n"
     "        if (fl >= nrh && fl < kRecW + nrh) __builtin_amdgcn_s_setprio(1);\n"
     "        const FrameHeadOut hd =\n"
     "            frame_head(c.sm, c.sV, c.sVG, fl * stride, lay.wcmax, rm, a.lambda, c.sRing + fl * kD * kD,\n"
     "                       c.sFlag + fl, f + 1,\n"
     "                       a.A_out && mine ? a.A_out + ((size_t)s * F + f) * kD * kD : nullptr,\n"
     "                       a.cost_out && mine ? a.cost_out + ((size_t)s * F + f) * kT * kT : nullptr,\n"
     "                       GRAD ? c.sCost + fl * kT * kT : nullptr, L, q, mine, fl >= nrh);\n"
     "        if (mine) {\n"
     "          if (L < kL && q < 2) {\n"
     "            float* m = c.sMring + fl * kL2 * kT;\n"
     "            *reinterpret_cast<float4*>(m + L * kT + 4 * q) = make_float4(hd.mT0[0], hd.mT0[1], hd.mT0[2], hd.mT0[3]);\n"
     "            *reinterpret_cast<float4*>(m + (kL + L) * kT + 4 * q) = make_float4(hd.mT1[0], hd.mT1[1], hd.mT1[2], hd.mT1[3]);\n"
     "          }\n"
     "          asm volatile(\"s_waitcnt lgkmcnt(0)\" ::: \"memory\");\n"
     "          if (lane == 0) lds_store_flag(c.sMflag + fl, f + 1);\n"
     "        }\n"
     "        __builtin_amdgcn_s_setprio(0);\n"
     "      }\n"
     "    }\n"
     "  }\n"
     "  for (int fb = 0; fb < c.nf; fb += lay.fc) {\n    const int cnt = (c.nf - fb) < lay.fc ? (c.nf - fb) : lay.fc;\n    if (fb > 0) {\n      scene_pos_dma<64 * (kRecW + NP)>"),
    ("    for (int i = pw; i < nh; i += NP) {\n      const int fl = hb + hs * i;",
     "    for (int i = pw + (fb == 0 ? peeled : 0); i < nh; i += NP) {\n      const int fl = hb + hs * i;"),
]
VARIANTS = {
    "base": {},
    "prev": {},   # prebuilt only: tools/ab/libg2k_prev.so (the last commit)
    "orig": {},
    "no_finalize": {SCENE: [("  poll_word(c.sTicket, NP + kRecW);\n  grad_priv_sum(c, NP);",
                             "  return;\n  poll_word(c.sTicket, NP + kRecW);\n  grad_priv_sum(c, NP);")]},
    "no_frame_grad": {SCENE: [("    frame_grad(a, lay, c, fl, dm, slot);", "")]},
    "no_tile_grad": {SCENE: [("  if (GRAD) {\n#pragma unroll\n    for (int v = 0; v < 4; ++v) {\n      d0[v] = has_t",
                              "  dWoT = f32x4{0.f, 0.f, 0.f, 0.f};\n  if (false) {\n#pragma unroll\n    for (int v = 0; v < 4; ++v) {\n      d0[v] = has_t")]},
    "stamps": {SCENE: STAMPS},
    "stamps_norecur": {SCENE: STAMPS + NO_RECUR},
    "nolsr": {"__flags__": ["-mllvm", "-disable-lsr"]},
    "no_recur": NO_RECUR_SCENE,
    "no_tiles": {SCENE: NO_TILES},
    "heads_first": {SCENE: HEADS_FIRST},
    "headprio2": {SCENE: [("      if (fl >= nrh && fl < NP + nrh) __builtin_amdgcn_s_setprio(1);   // the first round's heads",
                           "      if (fl >= nrh && fl < NP + nrh) __builtin_amdgcn_s_setprio(2);")]},
    "prio12": {SCENE: [("      if (fl >= nrh && fl < kRecW + nrh) __builtin_amdgcn_s_setprio(1);",
                        "      if (fl >= nrh && fl < NP + nrh) __builtin_amdgcn_s_setprio(1);")]},
    "prio_all": {SCENE: [("      if (fl >= nrh && fl < kRecW + nrh) __builtin_amdgcn_s_setprio(1);",
                          "      if (fl >= nrh) __builtin_amdgcn_s_setprio(1);")]},
    "prio_split": {SCENE: [("      if (fl >= nrh && fl < kRecW + nrh) __builtin_amdgcn_s_setprio(1);",
                            "      if (fl >= nrh) __builtin_amdgcn_s_setprio(fl < kRecW + nrh ? 2 : 1);")]},
    "tl_end_hf": {SCENE: lds_stamps(TL_END, head=False) + HEADS_FIRST},
    # output store cache policy (the product writes through: kStoreAux = 16, sc1)
    "st_plain": {"g2k_common.h": [("constexpr int kStoreAux = 16;", "constexpr int kStoreAux = 0;")]},
    "st_nt": {"g2k_common.h": [("constexpr int kStoreAux = 16;", "constexpr int kStoreAux = 2;")]},
    "st_sys": {"g2k_common.h": [("constexpr int kStoreAux = 16;", "constexpr int kStoreAux = 17;")]},
    "st_ntsc1": {"g2k_common.h": [("constexpr int kStoreAux = 16;", "constexpr int kStoreAux = 18;")]},
    "peel": {SCENE: PEEL},
    "tl_end_peel": {SCENE: lds_stamps(TL_END, head=False) + PEEL},
    "rec8": {SCENE: [("constexpr int kRecHeads = kRecW;", "constexpr int kRecHeads = 2 * kRecW;")]},
    "tl_end_rec8": {SCENE: lds_stamps(TL_END, head=False) + [("constexpr int kRecHeads = kRecW;", "constexpr int kRecHeads = 2 * kRecW;")]},
    "no_tile_mfma": {SCENE: [("      y0 = mfma4(a0[ks], w, y0);                           // Y[4q + v][n]\n      y1 = mfma4(L < kT ? a1[ks] : 0.f, w, y1);            // Y[16 + 4q + v][n] (0 for q >= 2)",
                              "      y0[0] = fmaf(a0[ks], w, y0[0]);\n      y1[0] = fmaf(a1[ks], w, y1[0]);")]},
    "no_m_mfma": {SCENE: [("      o.mT0 = mfma4(va[ks], bx[ks], o.mT0);   // M[L][4q+i]       (x rows)\n      o.mT1 = mfma4(va[ks], by[ks], o.mT1);   // M[12+L][4q+i]    (y rows)",
                           "      o.mT0[0] = fmaf(va[ks], bx[ks], o.mT0[0]);\n      o.mT1[0] = fmaf(va[ks], by[ks], o.mT1[0]);")]},
    "no_pred_store": {SCENE: [("      bstore(pr, n < nact ? (mrow(4 * q + v) * Nmax + n) * 4 : kBufOff, y0[v]);\n      bstore(pr, (n < nact && hi) ? (mrow(16 + 4 * q + v) * Nmax + n) * 4 : kBufOff, y1[v]);", "")]},
    "stamps_nolsr": {SCENE: STAMPS, "__flags__": ["-mllvm", "-disable-lsr"]},
    "stamps_tile": {SCENE: STAMPS + TILE},
    "stamps_fwd": {SCENE: STAMPS},
    "tl_fwd": {SCENE: TL_FWD},
    "tl_rec": {SCENE: TL_REC},
    "tl_lds": {SCENE: lds_stamps(TL_REC)},
    "tl_gap": {SCENE: lds_stamps(TL_REC + TL_GAP)},
    "tl_icache": {SCENE: lds_stamps(TL_REC + TL_ICACHE)},
    "tl_tile": {SCENE: lds_stamps(TL_REC + TL_TILE)},
    "tl_b1": {SCENE: lds_stamps(TL_B1 + TL_REC)},
    "pos1k": {SCENE: POS1K},
    "fullseg": {SCENE: [("    const bool okc = n0 + c4 < nact;", "    const bool okc = n0 + c4 < Nmax;")]},
    "zerotail": {SCENE: [("          load_item(fb, nitems, k + 3, tgB);\n        }\n      }\n    }\n",
        "          load_item(fb, nitems, k + 3, tgB);\n        }\n      }\n"
        "      if ((Nmax & 3) == 0) {\n"
        "        const int nz = c.ntiles - ntact;\n"
        "        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);\n"
        "        const int row = lane >> 2, c4 = 4 * (lane & 3);\n"
        "        for (int j = pw; j < cnt * nz; j += NP) {\n"
        "          const int fl = j / nz, t = ntact + (j - fl * nz), n0 = 16 * t;\n"
        "          const brsrc pr = make_brsrc(a.pred ? a.pred + ((size_t)s * F + fb + fl) * kL2 * Nmax : a.targets,\n"
        "                                      a.pred ? (uint32_t)kL2 * Nmax * 4 : 0u);\n"
        "          bstore4(pr, n0 + c4 < Nmax ? (row * Nmax + n0 + c4) * 4 : kBufOff, z4);\n"
        "          bstore4(pr, (n0 + c4 < Nmax && lane < 32) ? ((16 + row) * Nmax + n0 + c4) * 4 : kBufOff, z4);\n"
        "        }\n"
        "      }\n"
        "    }\n")]},
    "recprio1": {SCENE: [("      __builtin_amdgcn_s_setprio(2);\n      const float* as_lane", "      __builtin_amdgcn_s_setprio(1);\n      const float* as_lane")]},
    "recprio3": {SCENE: [("      __builtin_amdgcn_s_setprio(2);\n      const float* as_lane", "      __builtin_amdgcn_s_setprio(3);\n      const float* as_lane")]},
    "headprio": {SCENE: [("      if (fl < kRecW) __builtin_amdgcn_s_setprio(1);", "      __builtin_amdgcn_s_setprio(1);")]},
    # train mode at 16 waves (12 producers; the 128-VGPR cap spills)
    # LLVM scheduling strategies for the whole library
    "s_ilp": {"__flags__": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]},
    "s_memclause": {"__flags__": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"]},
    "s_trackers": {"__flags__": ["-mllvm", "-amdgpu-use-amdgpu-trackers"]},
    "np12t": {SCENE: [("  return grad ? 8 : 12;", "  return grad && H > 128 ? 8 : 12;"),
                      ("    if (NP == 8) {\n      switch (tpw) {\n        case 1: launch_k<1, 8, true>",
                       "    if (NP == 12 && tpw == 2) { launch_k<2, 12, true>(a, l, st); return G2K_OK; }\n    if (NP == 8) {\n      switch (tpw) {\n        case 1: launch_k<1, 8, true>")]},
    "np12": {SCENE: [("  return (H >= 256 || Nmax >= 64) ? 12 : 8;", "  return 12;")]},
    "np12ts": {SCENE: [("  return (H >= 256 || Nmax >= 64) ? 12 : 8;", "  return 12;"),
                       ("pred_tile<false, NP == 8>", "pred_tile<false, true>"),
                       ("o += grad ? NG * kL2 * kYP : (NP == 8 ? NP * kYS : 0);", "o += grad ? NG * kL2 * kYP : NP * kYS;")]},
    "lateloads": {SCENE: [("    } else {\n      load_item(fb, nitems, 0, tgA);\n      load_item(fb, nitems, 1, tgB);\n    }\n", "    }\n"),
                          ("      for (int k = 0; k < nitems; k += 2) {", "      load_item(fb, nitems, 0, tgA);\n      load_item(fb, nitems, 1, tgB);\n      for (int k = 0; k < nitems; k += 2) {")]},
    "prodsleep": {SCENE: [("        item(k, tgA);\n", "        item(k, tgA);\n        __builtin_amdgcn_s_sleep(2);\n")]},
    "tl_end": {SCENE: lds_stamps(TL_END, head=False)},
    "tl_end_orig": {SCENE: lds_stamps(TL_END, head=False)},
    "tl_b1_pos1k": {SCENE: lds_stamps(TL_B1 + TL_REC) + POS1K},
    "warm": {SCENE: WARM},
    "tl_lds_warm": {SCENE: lds_stamps(TL_REC) + WARM},
}
# variants of earlier experiments whose anchors no longer match the sources
# (their measurements are recorded in DESIGN.md §9 and profiles/): out of
# the runnable set until re-anchored
STALE = ('no_tile_grad', 'stamps', 'stamps_norecur', 'prio12', 'prio_all', 'prio_split',
         'rec8', 'tl_end_rec8', 'no_pred_store', 'stamps_nolsr', 'stamps_tile', 'stamps_fwd',
         'tl_tile', 'pos1k', 'fullseg', 'headprio', 'np12', 'np12ts', 'tl_b1_pos1k', 'warm', 'tl_lds_warm')
for _k in STALE:
    VARIANTS.pop(_k)


AB_DIR = os.path.join(ROOT, "tools", "ab")   # prebuilt variant libraries (git-ignored; travel to the box)


def variant_path(name):
    return os.path.join(AB_DIR, f"libg2k_{name}.so")


def build_variant(name):
    """Build variant `name` into tools/ab/libg2k_<name>.so (on the CPU host:
    the library travels to the GPU box with the tree)."""
    from concurrent.futures import ThreadPoolExecutor
    src = os.path.join(ROOT, "multimodaltraj_2_amd", "csrc")
    tmp = tempfile.mkdtemp(prefix=f"g2k_{name}_")
    for f in os.listdir(src):
        shutil.copy(os.path.join(src, f), tmp)
        if name == "orig" or name.endswith("_orig"):   # reference sources in tools/ab_ref (no .git on the box)
            ref = os.path.join(ROOT, "tools", "ab_ref", f)
            if os.path.exists(ref):
                shutil.copy(ref, os.path.join(tmp, f))
    for fname, reps in VARIANTS[name].items():
        if fname == "__flags__":
            continue
        p = os.path.join(tmp, fname)
        s = open(p).read()
        for a, b in reps:
            assert a in s, (name, a[:60])
            s = s.replace(a, b)
        if (name.startswith("stamps") or name.startswith("tl_")) and fname == SCENE:
            s += STAMP_EXPORT
        open(p, "w").write(s)
    os.makedirs(AB_DIR, exist_ok=True)
    out = variant_path(name)

    def comp(f):
        o = os.path.join(tmp, os.path.splitext(f)[0] + ".o")
        if f.endswith(".cpp"):
            cmd = [build.CXX, *build.CXX_FLAGS, "-c", "-o", o, os.path.join(tmp, f)]
        else:
            cmd = [build.HIPCC, *build.flags_for(f), *VARIANTS[name].get("__flags__", []), "-c", "-o", o,
                   os.path.join(tmp, f)]
        subprocess.run(cmd, check=True)
        return o

    files = sorted(f for f in os.listdir(tmp) if f.endswith(".hip") or f.endswith(".cpp"))
    with ThreadPoolExecutor(max_workers=8) as ex:
        objs = list(ex.map(comp, files))
    subprocess.run([build.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs],
                   check=True)
    shutil.rmtree(tmp, ignore_errors=True)
    return out


def variant_lib(name):
    """The prebuilt variant (tools/ab/), built here if missing (CPU host)."""
    p = variant_path(name)
    return p if os.path.exists(p) else build_variant(name)


def time_it(fn, reps=200, warm=20):
    for _ in range(warm):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def stamps(lib, c, t, dev, train=True):
    """Run the stamps build once and print scene 0's timeline (cycles)."""
    import ctypes
    import numpy as np
    params = fs.init_params(c["Nmax"], seed=0, device=dev)
    if train:
        plan = ts.TrainPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    else:
        plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
    S = t["pos"].shape[0]
    for _ in range(5):
        plan.run()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint * (S * 64))()
    assert lib.g2k_stamp_copy(buf, S * 64) == 0
    st = np.frombuffer(buf, dtype=np.uint32).reshape(S, 64).astype(np.int64)
    print("mode", "train" if train else "forward")
    for sc in (0, S // 2, S - 1):
        r = st[sc]
        rel = (r - r[0]) % (1 << 32)
        names = {21: "dma issue", 22: "pos dma issued", 23: "segs issued", 25: "nact loaded", 1: "B2",
                 2: "heads", 3: "tiles f0", 4: "tiles f1", 5: "tiles f2", 8: "fgrad f0",
                 9: "fgrad f1", 10: "fgrad f2", 12: "chunk sync", 13: "chunk sum", 14: "ticket",
                 15: "ticket=NP", 11: "priv summed", 16: "dWi done", 17: "prod start", 18: "dma waited",
                 19: "B1", 20: "recur end"}
        print(f"scene {sc} n_active {int(t['n_active'][sc])}: " +
              "  ".join(f"{v}:{rel[k]}" for k, v in names.items() if r[k] != 0))
        if train:
            print("   producers' tiles done:", " ".join(str(rel[24 + p]) for p in range(8)),
                  "(slot 25 collides in train mode)")
        print("   last tile 0 (poll, entry, Y, stores, err, dWoT, dM, dWo):", " ".join(str(rel[k]) for k in (46, 40, 41, 42, 43, 44, 45, 47)))
        print("   heads (start, head done, flags):", " ".join(f"({rel[30 + 3 * i]},{rel[31 + 3 * i]},{rel[32 + 3 * i]})" for i in range(3)))


def interleaved(cfg, names, rounds):
    """Plain variants timed in interleaved rounds (A B A B ...): per variant the
    median and min over rounds of the 200-launch HIP-event average."""
    import numpy as np
    c = dict(CONFIGS[cfg])
    S = c["S"] if c["S"] <= 256 else c["S"] // 8
    dev = torch.device("cuda")
    t = make_batch(S, c["Nmax"], c["H"], seed=1).to_device(dev)
    # as bench.py: n_frames and ped_mask bound; AB_ROTATE=K input batches in
    # rotation (no Infinity Cache hits), K = 1 by default
    K = int(os.environ.get("AB_ROTATE", "1"))
    batches = [t] + [make_batch(S, c["Nmax"], c["H"], seed=100 + k).to_device(dev) for k in range(1, K)]
    runs = {}
    for name in names:
        lib = _lib.load(variant_lib(name))
        _lib._lib = lib
        params = fs.init_params(c["Nmax"], seed=0, device=dev)
        plans = [fs.StepPlan(params, b["pos"], b["vislet"], b["G"], b["targets"], b["n_active"], b["h0"],
                             n_frames=b["n_frames"], ped_mask=b["ped_mask"]) for b in batches]
        tstep = ts.TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
        it = iter(range(1 << 62))
        runs[name] = (lib, (lambda ps=plans, it=it: ps[next(it) % len(ps)].run()), tstep)
    res = {n: ([], []) for n in names}
    for _ in range(rounds):
        for name in names:
            lib, run, tstep = runs[name]
            _lib._lib = lib
            res[name][0].append(time_it(run))
            res[name][1].append(time_it(tstep.run))
    for name in names:
        f, tr = np.array(res[name][0]), np.array(res[name][1])
        print(f"{cfg} {name:16s} fwd median {np.median(f):7.2f} min {f.min():7.2f}   "
              f"train median {np.median(tr):7.2f} min {tr.min():7.2f}  ({rounds} rounds)", flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--build":      # CPU host: prebuild the named variants
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=2) as ex:
            for out in ex.map(build_variant, [a for a in args[1:] if a in VARIANTS]):
                print(out)
        return
    if args and args[0] == "--rounds":
        rounds = int(args[1])
        rest = args[2:]
        cfg = rest[0] if rest and rest[0] in CONFIGS else "eth_hotel_synth"
        interleaved(cfg, [a for a in rest if a in VARIANTS], rounds)
        return
    cfg = args[0] if args and args[0] in CONFIGS else "eth_hotel_synth"
    names = [a for a in args if a in VARIANTS] or [v for v in VARIANTS if not v.startswith("stamps")]
    c = dict(CONFIGS[cfg])
    S = c["S"] if c["S"] <= 256 else c["S"] // 8
    dev = torch.device("cuda")
    b = make_batch(S, c["Nmax"], c["H"], seed=1)
    t = b.to_device(dev)
    for name in names:
        lib = _lib.load(variant_lib(name))
        _lib._lib = lib
        if name.startswith("tl_"):
            import numpy as np
            lib.g2k_stamp_copy.argtypes = [ctypes.c_void_p, ctypes.c_int]
            params = fs.init_params(c["Nmax"], seed=0, device=dev)
            # AB_ROTATE=K: the stamped launch reads inputs none of the K-1
            # launches before it touched (no Infinity Cache hits), as bench.py
            K = int(os.environ.get("AB_ROTATE", "0"))
            if K:
                plans = []
                for k in range(K):
                    tk = t if k == K - 1 else make_batch(S, c["Nmax"], c["H"], seed=100 + k).to_device(dev)
                    plans.append(fs.StepPlan(params, tk["pos"], tk["vislet"], tk["G"], tk["targets"],
                                             tk["n_active"], tk["h0"], n_frames=tk["n_frames"],
                                             ped_mask=tk["ped_mask"]))
                for p_ in plans:
                    p_.run()
                plan = plans[-1]
            else:
                plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
                for _ in range(5):
                    plan.run()
            torch.cuda.synchronize()
            W = 160 if name in ("tl_lds", "tl_gap", "tl_icache", "tl_lds_warm", "tl_tile", "tl_b1", "tl_b1_pos1k", "tl_end", "tl_end_orig", "tl_end_rec8", "tl_end_peel", "tl_end_hf") else 64
            buf = (ctypes.c_uint * (S * W))()
            assert lib.g2k_stamp_copy(buf, S * W) == 0
            st = np.frombuffer(buf, dtype=np.uint32).reshape(S, W).astype(np.int64)
            {"tl_fwd": tl_fwd_print, "tl_end": tl_end_print, "tl_end_orig": tl_end_print, "tl_end_rec8": tl_end_print, "tl_end_peel": tl_end_print, "tl_end_hf": tl_end_print}.get(name, tl_rec_print)(st, t)
            print(f"{name}: fwd {time_it(plan.run):7.2f} us (stamped build)")
            if name in ("tl_lds", "tl_gap", "tl_icache", "tl_lds_warm", "tl_tile", "tl_b1", "tl_b1_pos1k"):
                rel = (st - st[:, :1]) % (1 << 32)
                med = np.median(rel, axis=0)
                print("head 0 (median): operands", int(med[60]), "A done", int(med[61]), "attn done",
                      int(med[62]))
                if name.startswith("tl_b1"):
                    print("B1 waits per wave (median, wave 0..15):", [int(med[64 + w]) for w in range(16)])
                    print("wave starts (median, rel. to wave 0's stamp 0):", [int(med[80 + w]) for w in range(16)])
                    print("wave DMA issue start (median):", [int(med[96 + w]) for w in range(16)])
                    print("wave nact loaded (median):", [int(med[112 + w]) for w in range(16)])
                    print("wave at staging, before its DMA wait (median):", [int(med[128 + w]) for w in range(16)])
                if name == "tl_icache":
                    print("R0 head run twice (median): start", int(med[76]), "first done", int(med[77]),
                          "second done", int(med[78]))
                if name == "tl_gap":
                    print("P0 lead-in (median): B2", int(med[6]), "mask", int(med[70]), int(med[71]),
                          "targets issued", int(med[72]), "first head", int(med[7]), int(med[8]),
                          "second head", int(med[9]), int(med[10]),
                          "| R0 heads done", int(med[74]), "R0 chain start", int(med[75]))
                if name == "tl_tile":
                    print("last tile (median): entry", int(med[40]), "Y", int(med[41]), "targets", int(med[42]),
                          "stores", int(med[43]), "errors", int(med[44]))
            continue
        if name.startswith("stamps"):
            lib.g2k_stamp_copy.argtypes = [ctypes.c_void_p, ctypes.c_int]
            stamps(lib, c, t, dev, train=not name.endswith("_fwd"))
            continue
        params = fs.init_params(c["Nmax"], seed=0, device=dev)
        plan = fs.StepPlan(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"], t["h0"])
        tstep = ts.TrainStep(params, t["pos"], t["vislet"], t["G"], t["targets"], t["n_active"],
                             t["h0"])
        print(f"{cfg} {name:16s} fwd {time_it(plan.run):7.2f} us   train {time_it(tstep.run):7.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
