// g2k_recur.h — the attention + hidden-state recurrence of train.py:240-252
// held in MFMA registers (used by the fused scene kernel and by
// g2k_frame_recurrence_f32).
#pragma once
#include "g2k_common.h"

namespace g2k {

// ---------------------------------------------------------------------------
// Hidden recurrence (train.py:243-252), h in registers:
//   h <- softmax(h, -1); h <- As @ h; adj <- softmax(h, -1) @ 1; h <- adj * h
// computed as h' = (As diag(1/Z)) @ e with v_mfma_f32_16x16x4_f32 (M = the 16
// rows, N = 16 columns per tile, K = 16 in four k-steps), e = exp(h) and Z its
// row sums (softmax = e / Z).  Wave w owns columns [w*H/NW, (w+1)*H/NW) as TPW
// 16-wide tiles; lane (L = lane & 15, q = lane >> 4) holds rows 4q..4q+3 of
// column 16t + L: h'[4q + i][16t + L] in x[t][i].  That is the MFMA result
// layout and also exactly the B operand of the next frame's product
// (register ks = e[4q + ks][c]), so nothing is transposed between frames.  The
// A operand of lane (L, q) at k-step ks is As[L][4q + ks] / Z_{4q+ks}: one
// float4 of the As tile times the reciprocal row sums of the lane's own rows.
//
// Per frame: four MFMA k-steps per tile; e = exp(h'); per-row partial sums
// over the wave's columns (local + 16-lane DPP) published as one float4 per
// lane group; ONE NW-wave LDS exchange per frame (a workgroup barrier in
// g2k_recur_kernel, flag polling in the fused scene kernel).
//
// adj = sum_j softmax(h')_rj is evaluated from the published partials
// (sum_w P_w / Z) and scales the final h.  The next frame's softmax needs
// exp(adj * h'); |adj - 1| <= a few ulp (adj == 1 exactly in real arithmetic)
// and h' lies in [0, 1] (convex combinations of softmax outputs), so in fp32
// adj * h' is within one ulp of h' and exp(adj * h') is evaluated as
// exp(h') = e (DESIGN.md §6a "Recurrence numerics"); the same bound makes the
// tf.nn.softmax max shift the identity after frame 0.
// ---------------------------------------------------------------------------
template <int TPW, int NW>
struct Recur {
  static constexpr int kCols = 16 * TPW;   // columns per wave (H = NW * kCols)
  float x[TPW][4];    // h (before init) / the last h' (after a step)
  float e[TPW][4];    // exp(h'): numerators of the next softmax(h) = next B operand

  // rows >= D (D < 16: sample.py's num_freq_blocks) are held at zero
  __device__ __forceinline__ void load(const float* __restrict__ hs, int H, int wv, int q, int L,
                                       int D = kD) {
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        x[t][i] = (D == kD || 4 * q + i < D) ? hs[(4 * q + i) * H + wv * kCols + 16 * t + L] : 0.f;
  }

  // h = adj * h' with adj = row sum of softmax(h') from the last exchange
  // (red: that frame's [NW waves][16 rows] partials), or h unchanged (red NULL).
  __device__ __forceinline__ void store(float* __restrict__ hs, int H, int wv, int q, int L,
                                        const float* red, int D = kD) const {
    float adj[4] = {1.f, 1.f, 1.f, 1.f};
    if (red) {
      // after a step x holds h' * log2(e) (see body): adj carries the ln 2
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float z = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) z += red[16 * w + 4 * q + i];
        const float rz = rcp(z);
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) a = fmaf(red[16 * w + 4 * q + i], rz, a);
        adj[i] = a * kLn2;
      }
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (D == kD || 4 * q + i < D) hs[(4 * q + i) * H + wv * kCols + 16 * t + L] = adj[i] * x[t][i];
  }

  // softmax numerators of an arbitrary h (tf.nn.softmax max shift), in two
  // halves around a barrier the caller provides: the row max exchange, then
  // e and its row partials (published into red).
  __device__ __forceinline__ void init_max(float* mred, int wv, int q, int L) const {
    float m[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m[i] = x[0][i];
#pragma unroll
      for (int t = 1; t < TPW; ++t) m[i] = fmaxf(m[i], x[t][i]);
    }
    const float r = reduce4_rows16<true>(m[0], m[1], m[2], m[3], L);
    if (L < 4) mred[wv * 16 + 4 * q + reduce4_row(L)] = r;
  }
  __device__ __forceinline__ void init_exp(float* red, const float* mred, int wv, int q, int L) {
    float4 m = *reinterpret_cast<const float4*>(mred + 4 * q);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float4 v = *reinterpret_cast<const float4*>(mred + 16 * w + 4 * q);
      m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
    }
    const float mm[4] = {m.x, m.y, m.z, m.w};
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        e[t][i] = __expf(x[t][i] - mm[i]);
        p[i] += e[t][i];
      }
    publish(red, p, wv, q, L);
  }

  __device__ __forceinline__ void publish(float* red, float (&p)[4], int wv, int q, int L) const {
    const float r = reduce4_rows16<false>(p[0], p[1], p[2], p[3], L);
    if (L < 4) red[wv * 16 + 4 * q + reduce4_row(L)] = r;
  }

  // One frame with a workgroup barrier (g2k_recur_kernel).  b = As[L][4q..4q+3]
  // of this frame; red_cur: the row partials of e (previous exchange);
  // red_nxt: where this frame publishes its own.
  __device__ __forceinline__ void step(const float4 b, const float* red_cur, float* red_nxt,
                                       int wv, int q, int L) {
    float4 z = *reinterpret_cast<const float4*>(red_cur + 4 * q);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float4 v = *reinterpret_cast<const float4*>(red_cur + w * 16 + 4 * q);
      z.x += v.x; z.y += v.y; z.z += v.z; z.w += v.w;
    }
    const float zz[4] = {z.x, z.y, z.z, z.w};
    int dfl = 0;
    f32x4 dv = {0.f, 0.f, 0.f, 0.f};
    body<false>(make_float4(b.x * kLog2e, b.y * kLog2e, b.z * kLog2e, b.w * kLog2e),
                [&](int ks) { return zz[ks]; }, red_nxt, wv, q, L, dfl, dv);
    __syncthreads();
  }

  // One frame without a workgroup barrier (fused scene kernel): zq = the
  // previous exchange's row-partial quad of this lane's wave (poll_red), its
  // sums over the four waves formed by DPP when body needs them; after
  // publishing its row partials into red_nxt this wave raises its sequence
  // word.  pf_flag / pf_as: the next frame's As flag and row quad (read_as
  // order: flag, then data), issued before this frame's MFMA chain and waited
  // for after it, so their LDS latency hides under the chain.  The loads are
  // inline asm without their own wait; their registers are tied into the
  // waiting asm block ("+v"), which keeps the compiler from touching them in
  // between.
  __device__ __forceinline__ void step_seq(const float4 b, const f32x4 zq, float* red_nxt,
                                           int* seq, int seq_val, int wv, int q, int L,
                                           const int* pf_flag, const float* pf_as, int& pf_fl,
                                           float4& pf_b) {
    int fl;
    f32x4 v;
    asm volatile("ds_read_b32 %0, %2\n\tds_read_b128 %1, %3"
                 : "=&v"(fl), "=&v"(v)
                 : "v"(lds_addr(pf_flag)), "v"(lds_addr(pf_as))
                 : "memory");
    body<true>(b, [&](int ks) {   // lane L holds wave (L % NW)'s quad
      float t = zq[ks];
      t += dpp<0xB1>(t);   // quad_perm [1,0,3,2]
      t += dpp<0x4E>(t);   // quad_perm [2,3,0,1]
      if constexpr (NW == 8) t += dpp<0x124>(t);   // row_ror:4
      return t;
    }, red_nxt, wv, q, L, fl, v);
    asm volatile("" ::: "memory");   // partials land before the sequence word (LDS is in order)
    if ((threadIdx.x & 63) == 0) lds_store_flag(seq + wv, seq_val);
    pf_fl = fl;   // checked by the caller after its next poll
    pf_b = make_float4(v[0], v[1], v[2], v[3]);
  }

  // The A operand carries log2(e) (b = As * log2(e), scaled by whoever
  // stages As): the MFMA yields h' * log2(e) and the next numerators are exp2
  // of it directly (one v_exp_f32, no scaling multiply on the frame's
  // critical path); store() takes the ln 2 back.
  //
  // Issue order (the frame's critical path): the MFMAs go out by diagonals
  // d = t + ks (tile t, k-step ks), so tile 0 completes while the last
  // tiles' k-steps still run; a k-step's A operand b_ks / Z_ks is formed
  // under the MFMAs of the diagonal before it (z_of(ks) evaluated there), and
  // tile t's exp2 and row partials two diagonals after its last k-step (its
  // result has landed: 40-cycle dependent latency < two issues), under the
  // remaining MFMAs.  PF: wait for step_seq's prefetch (pf_fl, pf_v) after
  // the last MFMA is issued.
  template <bool PF, typename ZOf>
  __device__ __forceinline__ void body(const float4 b, ZOf z_of, float* red_nxt, int wv, int q,
                                       int L, int& pf_fl, f32x4& pf_v) {
    const float bb[4] = {b.x, b.y, b.z, b.w};
    float a[4];
    f32x4 acc[TPW];
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    auto finish = [&](int t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[t][i];
        x[t][i] = v;
        e[t][i] = __builtin_amdgcn_exp2f(v);    // h' in [0, 1]: no max shift needed
        p[i] += e[t][i];
      }
    };
    a[0] = bb[0] * rcp(z_of(0));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int d = 0; d < TPW + 3; ++d) {
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int ks = d - t;
        if (ks >= 0 && ks < 4)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ks], e[t][ks],
                                                        ks == 0 ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[t], 0, 0, 0);
      }
      if (d < 3) a[d + 1] = bb[d + 1] * rcp(z_of(d + 1));
      if (d >= 4 && d - 4 < TPW - 1) finish(d - 4);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (PF) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pf_fl), "+v"(pf_v)::"memory");
    finish(TPW - 1);   // (the loop finished tiles 0 .. TPW - 2)
    publish(red_nxt, p, wv, q, L);
  }
};

// ---------------------------------------------------------------------------
// The same recurrence with the product on split-f16 MFMAs (the fused scene
// kernel, D = 16).  v_mfma_f32_16x16x32_f16 takes 16 cycles per SIMD where
// the four k-steps of v_mfma_f32_16x16x4_f32 take 128 per tile; f16 carries
// 11 significant bits, so each f32 operand goes in as hi + lo (hi = the
// value rounded toward zero, lo = the f16 of the exact remainder: 22 bits)
// and a tile is TWO MFMAs over K = 32 slots (lane (L, q), slot j: row
// 4q + (j & 3) of the contraction):
//   A = {a_hi[0..3], a_lo[0..3]},  A' = {a_lo[0..3], a_hi[0..3]},
//   B = {b_hi[0..3], b_lo[0..3]}   (rows 4q..4q+3 of e, this lane's column)
//   A.B + A'.B = sum_rows (a_hi + a_lo)(b_hi + b_lo)
// (A and B index K by the same (lane group, slot), so the slot -> row map is
// free; A' is two 64-bit moves).  Products are exact in the f32
// accumulator; what the split loses is the rounding of each lo part, and
// every term is positive (As >= 0, e > 0).
//
// Range: the accumulator starts at -kOff (kOff = 7), so the exp2 of the
// result is e_s = 2^-7 e, its row sums Z_s = 2^-7 Z and the A operand
// b / Z_s = 128 As log2(e) / Z, with no scaling instruction anywhere.  The hi
// parts are f16 normals, but the lo parts mostly are NOT: e_s lies in
// [2^-7, 2^-5.6], so its lo part is below 2^-17 — an f16 subnormal, rounded
// to 2^-24 spacing, i.e. <= 2^-25 absolute (~2^-18 relative to e_s), and the
// same for the A operand's lo part.  The product's absolute error is then
// <= 2^-25 (sum_k A_k + 16 max e_s): ~3e-6 of h' at H = 128 and ~6e-6 at
// H = 512 in the worst case (all roundings aligned; DESIGN.md §6a
// "Recurrence numerics", measured 2.3e-6 at H 512 over 100 frames).  kOff = 7 balances the two terms for H = 128 .. 512
// (the optimum is 2^(2 kOff) ~ 30 Z): a smaller kOff shrinks the e term but
// grows the A term by the same factor.  close_h's 1e-5 bound is checked at
// H = 512 over 100 frames (tests/test_step_gpu.py); errors do not compound
// across frames (every frame renormalises).  The last frame starts its accumulator at 0 instead:
// its result is the output h' (an accumulator near -7 would hold h' log2(e)
// ~ 0.01 with 2^-22 absolute resolution only), and the adj ratio it feeds is
// scale-free.
// ---------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
constexpr float kOff = 7.f;

// hi (toward zero) and lo of four f32 values into the four dwords of an
// 8-slot f16 operand: {hi0 hi1 | hi2 hi3 | lo0 lo1 | lo2 lo3}.  lo = the f16
// of (v - hi) by v_fma_mix (one instruction per value, the difference exact
// in f32).
__device__ __forceinline__ u32x4v split4(float v0, float v1, float v2, float v3) {
  u32x4v o;
  o[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v0, v1));
  o[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(v2, v3));
  uint32_t l0, l1;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l0) : "v"(v0), "v"(o[0]));
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l1) : "v"(v2), "v"(o[1]));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l0) : "v"(v1), "v"(o[0]));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l1) : "v"(v3), "v"(o[1]));
  o[2] = l0;
  o[3] = l1;
  return o;
}

template <int TPW, int NW>
struct RecurH {
  static constexpr int kCols = 16 * TPW;   // columns per wave (H = NW * kCols)
  float x[TPW][4];    // h (before init) / the last accumulator (after a step)
  u32x4v bo[TPW];     // B of the next product: e_s of rows 4q..4q+3, hi then lo

  __device__ __forceinline__ void load(const float* __restrict__ hs, int H, int wv, int q, int L) {
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) x[t][i] = hs[(4 * q + i) * H + wv * kCols + 16 * t + L];
  }

  // h = adj * h' (adj from the last exchange's partials; red NULL: h as
  // loaded).  After a step x holds h' log2(e) (the last frame's accumulator
  // starts at 0): adj carries the ln 2.
  __device__ __forceinline__ void store(float* __restrict__ hs, int H, int wv, int q, int L,
                                        const float* red) const {
    float adj[4] = {1.f, 1.f, 1.f, 1.f};
    if (red) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float z = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) z += red[16 * w + 4 * q + i];
        const float rz = rcp(z);
        float a = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) a = fmaf(red[16 * w + 4 * q + i], rz, a);
        adj[i] = a * kLn2;
      }
    }
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) store_wt(hs + (4 * q + i) * H + wv * kCols + 16 * t + L, adj[i] * x[t][i]);
  }

  __device__ __forceinline__ void init_max(float* mred, int wv, int q, int L) const {
    float m[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m[i] = x[0][i];
#pragma unroll
      for (int t = 1; t < TPW; ++t) m[i] = fmaxf(m[i], x[t][i]);
    }
    const float r = reduce4_rows16<true>(m[0], m[1], m[2], m[3], L);
    if (L < 4) mred[wv * 16 + 4 * q + reduce4_row(L)] = r;
  }
  // softmax(h) numerators of the loaded h: e_s = 2^-kOff exp(h - max)
  __device__ __forceinline__ void init_exp(float* red, const float* mred, int wv, int q, int L) {
    float4 m = *reinterpret_cast<const float4*>(mred + 4 * q);
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const float4 v = *reinterpret_cast<const float4*>(mred + 16 * w + 4 * q);
      m.x = fmaxf(m.x, v.x); m.y = fmaxf(m.y, v.y); m.z = fmaxf(m.z, v.z); m.w = fmaxf(m.w, v.w);
    }
    const float mm[4] = {m.x, m.y, m.z, m.w};
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    float e[TPW][4];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        e[t][i] = __builtin_amdgcn_exp2f(fmaf(x[t][i] - mm[i], kLog2e, -kOff));
        p[i] += e[t][i];
      }
    publish(red, p, wv, q, L);
#pragma unroll
    for (int t = 0; t < TPW; ++t) bo[t] = split4(e[t][0], e[t][1], e[t][2], e[t][3]);
  }

  __device__ __forceinline__ void publish(float* red, float (&p)[4], int wv, int q, int L) const {
    const float r = reduce4_rows16<false>(p[0], p[1], p[2], p[3], L);
    if (L < 4) red[wv * 16 + 4 * q + reduce4_row(L)] = r;
  }

  // One frame (fused scene kernel; see Recur::step_seq for the exchange and
  // the prefetch): zq = the previous exchange's row-partial quad of this
  // lane's wave (lane L holds wave L % NW's), b = As[L][4q..4q+3] * log2(e)
  // of this frame, last: the scene's last frame (accumulator from 0).  The
  // B operands of the next frame are split after the sequence word is out.
  __device__ __forceinline__ void step_seq(const float4 b, const f32x4 zq, float* red_nxt,
                                           int* seq, int seq_val, int wv, int q, int L,
                                           const int* pf_flag, const float* pf_as, int& pf_fl,
                                           float4& pf_b, bool last) {
    int fl;
    f32x4 v;
    asm volatile("ds_read_b32 %0, %2\n\tds_read_b128 %1, %3"
                 : "=&v"(fl), "=&v"(v)
                 : "v"(lds_addr(pf_flag)), "v"(lds_addr(pf_as))
                 : "memory");
    float z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float t = zq[i];
      t += dpp<0xB1>(t);                     // quad_perm [1,0,3,2]
      t += dpp<0x4E>(t);                     // quad_perm [2,3,0,1]
      if constexpr (NW == 8) t += dpp<0x124>(t);   // row_ror:4 (the other quad's four waves)
      z[i] = t;
    }
    const u32x4v A = split4(b.x * rcp(z[0]), b.y * rcp(z[1]), b.z * rcp(z[2]), b.w * rcp(z[3]));
    const u32x4v A2 = {A[2], A[3], A[0], A[1]};
    const float c0 = last ? 0.f : -kOff;
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, A), __builtin_bit_cast(f16x8, bo[t]),
                                                      f32x4{c0, c0, c0, c0}, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TPW; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, A2), __builtin_bit_cast(f16x8, bo[t]),
                                                      acc[t], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fl), "+v"(v)::"memory");
    float e[TPW][4];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[t][i] = acc[t][i];
        e[t][i] = __builtin_amdgcn_exp2f(acc[t][i]);   // 2^-7 exp(h') (h' in [0, 1]: no max shift)
      }
    float p[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p[i] = e[0][i];
#pragma unroll
      for (int t = 1; t < TPW; ++t) p[i] += e[t][i];
    }
    publish(red_nxt, p, wv, q, L);
    asm volatile("" ::: "memory");   // partials land before the sequence word (LDS is in order)
    if ((threadIdx.x & 63) == 0) lds_store_flag(seq + wv, seq_val);
#pragma unroll
    for (int t = 0; t < TPW; ++t) bo[t] = split4(e[t][0], e[t][1], e[t][2], e[t][3]);
    pf_fl = fl;
    pf_b = make_float4(v[0], v[1], v[2], v[3]);
  }
};

}  // namespace g2k
