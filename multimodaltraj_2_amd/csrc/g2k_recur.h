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
// exp(h') = e (DESIGN.md "recurrence numerics"); the same bound makes the
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
    int dfl = 0;
    f32x4 dv = {0.f, 0.f, 0.f, 0.f};
    body<false>(make_float4(b.x * kLog2e, b.y * kLog2e, b.z * kLog2e, b.w * kLog2e), z, red_nxt, wv, q,
                L, dfl, dv);
    __syncthreads();
  }

  // One frame without a workgroup barrier (fused scene kernel): z was polled
  // from the previous exchange (poll_red); after publishing its row partials
  // into red_nxt this wave raises its sequence word.  pf_flag / pf_as: the
  // next frame's As flag and row quad (read_as order: flag, then data),
  // issued before this frame's MFMA chain and waited for after it, so their
  // LDS latency hides under the chain.  The loads are inline asm without
  // their own wait; their registers are tied into the waiting asm block
  // ("+v"), which keeps the compiler from touching them in between.
  __device__ __forceinline__ void step_seq(const float4 b, const float4 z, float* red_nxt,
                                           int* seq, int seq_val, int wv, int q, int L,
                                           const int* pf_flag, const float* pf_as, int& pf_fl,
                                           float4& pf_b) {
    int fl;
    f32x4 v;
    asm volatile("ds_read_b32 %0, %2\n\tds_read_b128 %1, %3"
                 : "=&v"(fl), "=&v"(v)
                 : "v"(lds_addr(pf_flag)), "v"(lds_addr(pf_as))
                 : "memory");
    body<true>(b, z, red_nxt, wv, q, L, fl, v);
    asm volatile("" ::: "memory");   // partials land before the sequence word (LDS is in order)
    if ((threadIdx.x & 63) == 0) lds_store_flag(seq + wv, seq_val);
    pf_fl = fl;   // checked by the caller after its next poll
    pf_b = make_float4(v[0], v[1], v[2], v[3]);
  }

  // The A operand carries log2(e) (b = As * log2(e), scaled by whoever
  // stages As): the MFMA yields h' * log2(e) and the next numerators are exp2
  // of it directly (one v_exp_f32, no scaling multiply on the frame's
  // critical path); store() takes the ln 2 back.  PF: wait for step_seq's
  // prefetch (pf_fl, pf_v) right after the MFMA chain is issued.
  template <bool PF = false>
  __device__ __forceinline__ void body(const float4 b, const float4 z, float* red_nxt, int wv,
                                       int q, int L, int& pf_fl, f32x4& pf_v) {
    const float a0 = b.x * rcp(z.x);
    const float a1 = b.y * rcp(z.y);
    const float a2 = b.z * rcp(z.z);
    const float a3 = b.w * rcp(z.w);
    __builtin_amdgcn_sched_barrier(0);   // MFMAs back to back, k-step major
    f32x4 acc[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, e[t][0], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, e[t][1], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a2, e[t][2], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a3, e[t][3], acc[t], 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);
    if (PF) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pf_fl), "+v"(pf_v)::"memory");
    float p[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[t][i];
        x[t][i] = v;
        e[t][i] = __builtin_amdgcn_exp2f(v);    // h' in [0, 1]: no max shift needed
        p[i] += e[t][i];
      }
    publish(red_nxt, p, wv, q, L);
  }
};

}  // namespace g2k
