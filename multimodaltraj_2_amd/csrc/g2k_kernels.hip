// g2k_kernels.hip — gfx950 (CDNA4) kernels + C ABI for the g2k_lstm_mcr
// per-frame path of serenetech90/multimodaltraj_2.
//
//   g2k_scene_kernel — the step (train.py:197-276 over S scenes x F frames) in
//      ONE launch: one workgroup per scene; producer waves run the frame heads
//      (a2-a7), predictions and a9 errors per frame, recurrence waves run a8
//      with h [16, H] in MFMA registers; LDS flags between them, barriers
//      only at chunk boundaries.
//   g2k_frames_kernel + g2k_recur_kernel — the earlier two-kernel split
//      (G2K_STEP_SPLIT=1, g2k_frame_recurrence_f32).
//   g2k_mcr_forward_kernel, g2k_errors_v0/v1_kernel, relation ops (a7, a9, a11).
//   g2k_gridlstm_kernel — GridLSTMCell encoders (a6).
//   g2k_grad_kernel + reductions + g2k_update_kernel — train mode.
//   g2k_ctx_conv_kernel + g2k_ctx_reduce_kernel — static-context input (a5).
// Deterministic: fixed reduction order, no float atomics.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#include "g2k_hip.h"

namespace {

constexpr int kT = 8;     // obs_len
constexpr int kL = 12;    // pred_len
constexpr int kL2 = 24;   // 2 * pred_len rows of temp_path
constexpr int kD = 16;    // hidden_len
constexpr int kNT = 256;  // threads per workgroup
constexpr int kMaxN = 256;
constexpr int kRecurChunk = 32;         // As tiles resident in LDS in g2k_recur_kernel

thread_local char g_err[512] = "";

int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_err(G2K_ELAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
  return G2K_OK;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

#ifdef G2K_STAMPS
// diagnostic build only: s_memtime stamps of workgroup 0 of each kernel
__device__ unsigned long long g2k_stamps[64];
#define STAMP(k)                                                              \
  do {                                                                        \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0 && (k) < 64)   \
      g2k_stamps[(k)] = __builtin_amdgcn_s_memtime();                         \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

#ifdef G2K_STAMPS_SCENE
// diagnostic build only: timeline of scene-kernel workgroups 0, 85, 170, 255.
// Stamps are s_memtime (shader clock, low 32 bits) kept in LDS and copied
// out at the end, so they do not perturb the vmcnt accounting of the code
// around them (each still waits lgkmcnt(0) for its own value).
__device__ unsigned g2k_sstamps[4][128];
__shared__ unsigned g2k_lds_stamps[128];
#define SSTAMP(k, cond)                                                         \
  do {                                                                          \
    if (cond) {                                                                 \
      unsigned long long _t;                                                    \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory"); \
      g2k_lds_stamps[(k)] = (unsigned)_t;                                       \
    }                                                                           \
  } while (0)
#define SSTAMP_FLUSH()                                                          \
  do {                                                                          \
    __syncthreads();                                                            \
    if ((blockIdx.x % 85) == 0 && blockIdx.x < 340 && threadIdx.x < 128)       \
      g2k_sstamps[blockIdx.x / 85][threadIdx.x] = g2k_lds_stamps[threadIdx.x];  \
  } while (0)
#define SSTAMP_INIT()                                                           \
  do {                                                                          \
    if (threadIdx.x < 128) g2k_lds_stamps[threadIdx.x] = 0xFFFFFFFFu;           \
  } while (0)
#else
#define SSTAMP(k, cond) do {} while (0)
#define SSTAMP_FLUSH() do {} while (0)
#define SSTAMP_INIT() do {} while (0)
#endif


__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// The wave's index in its workgroup, provably wave-uniform (an SGPR): role
// branches, per-wave loops and s_setprio guards on it compile to scalar
// branches instead of exec-masked code.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }


// LDS-DMA: 16 bytes per lane, LDS destination = wave-uniform base + 16*lane.
__device__ __forceinline__ void dma16(const float* gsrc, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

// Copy n4 float4s (contiguous, 16-B aligned) global -> LDS with a workgroup
// of NT threads; the caller waits (vmcnt(0)) and barriers before reading.
template <int NT>
__device__ __forceinline__ void dma_copy_n(const float* g, float* lds, int n4, int wv, int lane) {
  for (int i = wv * 64; i < n4; i += NT) {
    if (i + lane < n4) dma16(g + (size_t)(i + lane) * 4, lds + i * 4);
  }
}

// Copy n floats global -> LDS with the whole workgroup by 4-byte LDS-DMA
// (no alignment requirement beyond 4 bytes); caller waits vmcnt(0) + barrier.
template <int NT>
__device__ __forceinline__ void dma4_copy_t(const float* g, float* lds, int n, int wv, int lane) {
  for (int i = wv * 64; i < n; i += NT) {
    if (i + lane < n)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + i + lane),
                                       (__attribute__((address_space(3))) void*)(lds + i), 4, 0, 0);
  }
}

__device__ __forceinline__ void dma4_copy(const float* g, float* lds, int n, int wv, int lane) {
  for (int i = wv * 64; i < n; i += kNT) {
    if (i + lane < n)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + i + lane),
                                       (__attribute__((address_space(3))) void*)(lds + i), 4, 0, 0);
  }
}

// ---------------------------------------------------------------------------
// wave-level helpers
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 16 lanes of a DPP row; every lane of the row gets the result.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}


// Sum over the four 16-lane rows of a wave (lanes r, r+16, r+32, r+48),
// identical bits in all four lanes: v_permlane32_swap + v_permlane16_swap.
__device__ __forceinline__ float sum_rows4(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Sum over all 64 lanes (DPP + permlane, no LDS); every lane gets the result.
__device__ __forceinline__ float wave_sum(float v) { return sum_rows4(row16_sum(v)); }

// Four per-lane values v[i] (rows 4q + i of an MFMA result, this lane's
// column) reduced over the 16 lanes of each lane group by a transposing
// butterfly: 2 + 1 DPP exchanges hand each lane one row, 2 more finish the
// row.  Lane L ends with the reduction of row 4q + reduce4_row(L).
__device__ __forceinline__ int reduce4_row(int L) { return 2 * (L & 1) + ((L >> 1) & 1); }

template <bool MAX>
__device__ __forceinline__ float reduce4_rows16(float v0, float v1, float v2, float v3, int L) {
  auto op = [](float x, float y) { return MAX ? fmaxf(x, y) : x + y; };
  const bool odd = (L & 1) != 0, b1 = (L & 2) != 0;
  const float s0 = odd ? v0 : v2, s1 = odd ? v1 : v3;        // rows the xor-1 partner keeps
  const float a0 = op(odd ? v2 : v0, dpp<0xB1>(s0));        // quad_perm [1,0,3,2]
  const float a1 = op(odd ? v3 : v1, dpp<0xB1>(s1));
  float r = op(b1 ? a1 : a0, dpp<0x4E>(b1 ? a0 : a1));      // quad_perm [2,3,0,1]
  r = op(r, dpp<0x124>(r));                                 // row_ror:4
  r = op(r, dpp<0x128>(r));                                 // row_ror:8
  return r;
}

// ---------------------------------------------------------------------------
// a9 error terms for one (frame, pedestrian): y = pred_path_band[:, n] as 24
// rows (x rows 0..11, y rows 12..23), tgt = 12 (x, y) pairs (16-B aligned).
// train.py:640-656: ade_i = ||P_[i][:L] - tgt[:L]||_2 (spectral) / 12,
//                   err = P_[i][L-1] - tgt[L-1]  (fde vector).
// acc: {ade_spec, count, |fde|^2, ade_l2, |fde|}
// ---------------------------------------------------------------------------
__device__ __forceinline__ void error_terms(const float* y, const float* tgt, float acc[5]) {
  const float4* t4 = reinterpret_cast<const float4*>(tgt);
  float tv[kL2];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    float4 v = t4[k];
    tv[4 * k + 0] = v.x; tv[4 * k + 1] = v.y; tv[4 * k + 2] = v.z; tv[4 * k + 3] = v.w;
  }
  float a = 0.f, b = 0.f, c = 0.f, l2 = 0.f;
  float fx = 0.f, fy = 0.f;
#pragma unroll
  for (int l = 0; l < kL; ++l) {
    const float dx = y[l] - tv[2 * l];
    const float dy = y[kL + l] - tv[2 * l + 1];
    a = fmaf(dx, dx, a);
    b = fmaf(dx, dy, b);
    c = fmaf(dy, dy, c);
    l2 += sqrtf(fmaf(dx, dx, dy * dy));
    fx = dx; fy = dy;
  }
  // largest singular value of the [L, 2] difference: sqrt(lambda_max(M^T M))
  const float hm = 0.5f * (a - c);
  const float lam = 0.5f * (a + c) + sqrtf(fmaf(hm, hm, b * b));
  const float fsq = fmaf(fx, fx, fy * fy);
  acc[0] += sqrtf(fmaxf(lam, 0.f)) * (1.0f / 12.0f);
  acc[1] += 1.0f;
  acc[2] += fsq;
  acc[3] += l2 * (1.0f / 12.0f);
  acc[4] += sqrtf(fsq);
}

// ---------------------------------------------------------------------------
// As = softmax(exp(A) / cumsum(exp(A), axis=0), axis=-1)   (train.py:240)
// Column pass with a running max so exp never overflows (the ratio
// exp(a_r) / sum_{k<=r} exp(a_k) is scale-invariant), then a row softmax of
// values in (0, 1].  `A` is one [16, 16] tile in LDS, transformed in place.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void attn_column_pass(float* A, int c) {
  float m = -INFINITY, s = 0.f;
#pragma unroll
  for (int r = 0; r < kD; ++r) {
    const float a = A[r * kD + c];
    const float mn = fmaxf(m, a);
    const float ea = __expf(a - mn);
    s = fmaf(s, __expf(m - mn), ea);
    m = mn;
    A[r * kD + c] = ea * rcp(s);
  }
}

__device__ __forceinline__ void attn_row_pass(float* A, int r, float* gout) {
  float4* row = reinterpret_cast<float4*>(A + r * kD);
  float e[kD];
  float z = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float4 v = row[k];
    e[4 * k + 0] = __expf(v.x); e[4 * k + 1] = __expf(v.y);
    e[4 * k + 2] = __expf(v.z); e[4 * k + 3] = __expf(v.w);
  }
#pragma unroll
  for (int k = 0; k < kD; ++k) z += e[k];
  const float rz = rcp(z);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float4 v = make_float4(e[4 * k] * rz, e[4 * k + 1] * rz, e[4 * k + 2] * rz, e[4 * k + 3] * rz);
    row[k] = v;
    if (gout) reinterpret_cast<float4*>(gout + r * kD)[k] = v;
  }
}


// ---------------------------------------------------------------------------
// LDS polling for the wave-specialised scene kernel.  The loads are inline
// asm (the compiler may neither hoist nor merge them) and wait for their own
// data; LDS services one CU's requests in order, so a flag read that sees a
// producer's flag write is followed by data reads that see the data the
// producer wrote before it (the producer waits lgkmcnt(0) between the two).
// A poll gives up after kPollMax rounds (~50 ms) so that a broken invariant
// yields wrong numbers, not a hung GPU.
// ---------------------------------------------------------------------------
constexpr int kPollMax = 1 << 20;
#ifndef G2K_POLL_SLEEP
#define G2K_POLL_SLEEP 1
#endif

__device__ __forceinline__ void poll_pause() {
  if (G2K_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(G2K_POLL_SLEEP);
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Flag / sequence-word store: a plain ds_write_b32 (a volatile store through a
// generic pointer compiles to a flat store + vmcnt(0) wait, hundreds of cycles
// on the critical path).  Ordered after the caller's earlier LDS writes by the
// in-order LDS queue; the memory clobber keeps the compiler from sinking them.
__device__ __forceinline__ void lds_store_flag(int* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}



// The recurrence's per-frame exchange, split in two LDS round trips so that
// the one on the critical path is small:
//  - read_as: the producer's flag of a frame's As tile, then the lane's As
//    row quad (As[L][4q..4q+3]), one asm block (LDS serves a CU's requests in
//    order and the producer stores the tile before the flag, so a current
//    flag means a current quad).  Issued right after the previous frame's
//    publish, while the other waves are still finishing theirs.
//  - poll_red: spin on ONE wave's sequence word (lane L reads wave L & 3's:
//    seq[w] = frames whose partials w has published, +1) together with that
//    wave's row-partial quad of rows 4q..4q+3; the four waves' quads are then
//    summed across each lane quad by DPP.  Data is stored before the word and
//    read after it, so a current word means current data.
// Busy poll for the first rounds, then s_sleep.
__device__ __forceinline__ int read_as(const int* flag, const float* asrc, float4& b) {
  const uint32_t fa = lds_addr(flag), da = lds_addr(asrc);
  int fl;
  f32x4 v;
  asm volatile(
      "ds_read_b32 %0, %2\n\t"
      "ds_read_b128 %1, %3\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(fl), "=&v"(v)
      : "v"(fa), "v"(da)
      : "memory");
  b = make_float4(v[0], v[1], v[2], v[3]);
  return __builtin_amdgcn_readfirstlane(fl);
}

// Slow path of read_as: the tile was not ready when first read.
__device__ __forceinline__ void wait_as(const int* flag, int want, const float* asrc, float4& b) {
  for (int it = 0; it < kPollMax; ++it) {
    if (read_as(flag, asrc, b) == want) break;
    if (it >= 8) __builtin_amdgcn_s_sleep(1);   // long waits (the first heads): back off
  }
}

__device__ __forceinline__ void poll_red(const int* seq_w, int want_seq, const float* rslot,
                                         float4& z) {
  const uint32_t sa = lds_addr(seq_w), ra = lds_addr(rslot);
  int sq;
  f32x4 r;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile(
        "ds_read_b32 %0, %2\n\t"
        "ds_read_b128 %1, %3\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(sq), "=&v"(r)
        : "v"(sa), "v"(ra)
        : "memory");
    if (__builtin_amdgcn_ballot_w64(sq < want_seq) == 0) break;
    if (it >= 8) __builtin_amdgcn_s_sleep(1);
  }
  float zz[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float t = r[i];
    t += dpp<0xB1>(t);   // quad_perm [1,0,3,2]
    t += dpp<0x4E>(t);   // quad_perm [2,3,0,1]
    zz[i] = t;
  }
  z = make_float4(zz[0], zz[1], zz[2], zz[3]);
}

// Wait until all four recurrence waves' sequence words reach `want`.
__device__ __forceinline__ void poll_seq_all(const int* seq, int want) {
  const uint32_t sa = lds_addr(seq);
  i32x4 sq;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(sq) : "v"(sa) : "memory");
    const int mn = min(min(sq[0], sq[1]), min(sq[2], sq[3]));
    if (__builtin_amdgcn_readfirstlane(mn) >= want) break;
  }
}

// Wait until every lane's sequence word (lane L reads seq_w = seq + (L & 3))
// reaches `want`.
__device__ __forceinline__ void poll_seq(const int* seq_w, int want) {
  const uint32_t sa = lds_addr(seq_w);
  int sq;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(sq) : "v"(sa) : "memory");
    if (__builtin_amdgcn_ballot_w64(sq < want) == 0) break;
  }
}

// Wait until a frame flag reaches `want` (no data attached).
__device__ __forceinline__ void poll_flag(const int* flag, int want) {
  const uint32_t fa = lds_addr(flag);
  int fl;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(fl) : "v"(fa) : "memory");
    if (__builtin_amdgcn_readfirstlane(fl) == want) break;
    poll_pause();
  }
}

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

  __device__ __forceinline__ void load(const float* __restrict__ hs, int H, int wv, int q, int L) {
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) x[t][i] = hs[(4 * q + i) * H + wv * kCols + 16 * t + L];
  }

  // h = adj * h' with adj = row sum of softmax(h') from the last exchange
  // (red: that frame's [NW waves][16 rows] partials), or h unchanged (red NULL).
  __device__ __forceinline__ void store(float* __restrict__ hs, int H, int wv, int q, int L,
                                        const float* red) const {
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
      for (int i = 0; i < 4; ++i) hs[(4 * q + i) * H + wv * kCols + 16 * t + L] = adj[i] * x[t][i];
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

// ---------------------------------------------------------------------------
// Kernel 1: frame-parallel part.  One workgroup = 4 waves = kFramesPerWG
// consecutive frames of one scene; one wave computes one frame.
//
// The workgroup stages the weights, lambda*G and the norms of its position
// window in LDS and forms V = norms @ Wi for every window row (+ the two
// vislet rows Ve) cooperatively; after that barrier every wave runs its frame
// alone.  All the frame's small matmuls are v_mfma_f32_16x16x4_f32 chained in
// registers: for D = A @ B the A operand of lane (L = lane & 15, q = lane >> 4)
// at k-step ks is A[L][k], the B operand B[k][L], with k = 4q + ks, and the
// result lands as D[4q + i][L] in register i — i.e. register ks of one result
// is exactly the k-step-ks operand of a product that contracts over its row
// index.  Each product below is oriented so that this holds:
//   X0   = Wii @ U                       (U = V rows of the window)
//   E    = Wv[:, :16] @ X0  (+ Ec + bv)  rows t on the lane group
//   E^T  = X0^T @ Wv[:, :16]^T           rows t on the lane
//   A    = g @ (E * Rm)                  -> As (train.py:240) -> workspace
//   cost = E @ g
//   M^T  = cost^T @ Wc^T   (x rows, y rows as two 16-wide tiles)
//   Y^T  = Wo^T @ M^T      per 16 pedestrians -> pred_path_band, errors
// (8-wide contractions use k-steps with zero rows: t = 4q + ks < 8.)
// ---------------------------------------------------------------------------
constexpr int kFramesPerWG = 4;

struct FrameLayout {
  int np;   // padded norm row stride
  int o_wi, o_wo, o_nrm, o_v, o_small, o_y, o_pos, o_met;
  int total;
};

__host__ __device__ inline int rup4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline FrameLayout frame_layout(int Nmax, int stride) {
  FrameLayout s;
  const int wc = (kFramesPerWG - 1) * stride + kT;
  s.np = Nmax + 1;
  int o = 0;
  s.o_wi = o;    o += rup4(Nmax * kD);
  s.o_wo = o;    o += rup4(kT * Nmax);
  s.o_nrm = o;   o += rup4((wc + 2) * s.np);
  s.o_v = o;     o += rup4((wc + 2) * kD);
  s.o_small = o; o += 1024;
  s.o_y = o;     o += 4 * kD * kL2;         // per-wave prediction transpose [16 peds][12][2]
  s.o_pos = o;   o += rup4(wc * Nmax * 2);  // raw position window (LDS-DMA)
  s.o_met = o;   o += 64;
  s.total = o;
  return s;
}

// offsets inside the `small` block
constexpr int SM_WII = 0;     // [16][8]
constexpr int SM_WV = 128;    // [8][18]  (144)
constexpr int SM_BV = 272;    // [16]
constexpr int SM_WR = 288;    // [8][2]
constexpr int SM_WC = 304;    // [24][8]  (192)
constexpr int SM_G = 496;     // [16][8]  lambda * G
// end 624 <= 1024

struct StepArgs {
  g2k_dims d;
  g2k_weights w;
  const float* pos;
  const float* vislet;
  const float* G;
  const float* targets;
  const int32_t* n_active;
  const int32_t* n_frames;
  const uint8_t* ped_mask;
  const float* h_in;
  float* h_out;
  float* pred;
  float* metrics;
  float* A_out;
  float* cost_out;
  float* ws_as;        // [S, F, 16, 16] attention weights
  float* ws_part;      // [S, nchunk, 8] ADE/FDE partial sums
  float lambda;
  int nchunk;
  int dma16;           // scene kernel: every input 16-B aligned and Nmax even (16-byte LDS-DMA)
  int opts;            // scene kernel options (kOpt*)
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// online (max, sum-of-exp) pair combine
__device__ __forceinline__ void lse_combine(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

__global__ void __launch_bounds__(kNT) g2k_frames_kernel(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int chunk = blockIdx.x, s = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), L = lane & 15, q = lane >> 4;
  const int Nmax = a.d.Nmax, W = a.d.W, F = a.d.F, stride = a.d.stride;
  const int nact = clampi(a.n_active[s], 0, Nmax);
  const int nf = a.n_frames ? clampi(a.n_frames[s], 0, F) : F;
  const int f0 = chunk * kFramesPerWG;
  float* part = a.ws_part + ((size_t)s * a.nchunk + chunk) * 8;
  STAMP(0);

  // frames of this chunk beyond n_frames: zero predictions
  {
    const int z0 = f0 > nf ? f0 : nf;
    const int z1 = (f0 + kFramesPerWG) < F ? (f0 + kFramesPerWG) : F;
    for (int i = tid; i < (z1 - z0) * kL2 * Nmax; i += kNT)
      a.pred[((size_t)s * F + z0) * kL2 * Nmax + i] = 0.f;
  }
  if (f0 >= nf) {                       // uniform per workgroup
    if (tid < 8) part[tid] = 0.f;
    return;
  }
  const int fa = (nf - f0) < kFramesPerWG ? (nf - f0) : kFramesPerWG;
  const int r0 = f0 * stride, wc = (fa - 1) * stride + kT;
  const FrameLayout lay = frame_layout(Nmax, stride);
  // this wave's first-tile targets go in flight before the staging
  float2 tgA[3] = {};
  if (wv < fa) {
    const int pp0 = lane >> 2, u0 = lane & 3;
    const float2* tp = reinterpret_cast<const float2*>(
        a.targets + (((size_t)s * F + f0 + wv) * Nmax + (pp0 < Nmax ? pp0 : 0)) * kL2) + 3 * u0;
    tgA[0] = tp[0]; tgA[1] = tp[1]; tgA[2] = tp[2];
  }
  float* sWi = smem + lay.o_wi;
  float* sWo = smem + lay.o_wo;
  float* sNrm = smem + lay.o_nrm;
  float* sV = smem + lay.o_v;
  float* sm = smem + lay.o_small;
  float* sMet = smem + lay.o_met;
  float* sPos = smem + lay.o_pos;
  const int np = lay.np;

  // ---- staging by LDS-DMA (dword granules: any alignment), one wait -------
  {
    dma4_copy(a.w.Wi, sWi, Nmax * kD, wv, lane);
    dma4_copy(a.w.Wo, sWo, kT * Nmax, wv, lane);
    dma4_copy(a.w.Wii, sm + SM_WII, kD * kT, wv, lane);
    dma4_copy(a.G + (size_t)s * kD * kT, sm + SM_G, kD * kT, wv, lane);
    dma4_copy(a.w.Wv, sm + SM_WV, kT * (kD + 2), wv, lane);
    dma4_copy(a.w.bv, sm + SM_BV, kD, wv, lane);
    dma4_copy(a.w.Wr, sm + SM_WR, kT * 2, wv, lane);
    dma4_copy(a.w.Wc, sm + SM_WC, kL2 * kT, wv, lane);
    const float* vis = a.vislet + (size_t)s * 2 * Nmax;
    dma4_copy(vis, sNrm + wc * np, Nmax, wv, lane);
    dma4_copy(vis + Nmax, sNrm + (wc + 1) * np, Nmax, wv, lane);
    dma4_copy(a.pos + ((size_t)s * W + r0) * Nmax * 2, sPos, wc * Nmax * 2, wv, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // window norms ||(x, y)||_2 (train.py:79); ngh = lambda * ngh (g2k_lstm_mcr.py:102)
  for (int i = tid; i < wc * Nmax; i += kNT) {
    const int w = i / Nmax, n = i - w * Nmax;
    const float2 p = reinterpret_cast<const float2*>(sPos)[i];
    sNrm[w * np + n] = n < nact ? sqrtf(fmaf(p.x, p.x, p.y * p.y)) : 0.f;
  }
  if (tid < kD * kT) sm[SM_G + tid] *= a.lambda;
  __syncthreads();
  STAMP(1);
  // ---- V = norms @ Wi (train.py:179 for every window row) and Ve rows -----
  {
    const int dcol = tid & 15;
    for (int w = tid >> 4; w < wc + 2; w += kNT / 16) {
      const float* nr = sNrm + w * np;
      float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
      int n = 0;
      for (; n + 4 <= nact; n += 4) {
        acc0 = fmaf(nr[n], sWi[n * kD + dcol], acc0);
        acc1 = fmaf(nr[n + 1], sWi[(n + 1) * kD + dcol], acc1);
        acc2 = fmaf(nr[n + 2], sWi[(n + 2) * kD + dcol], acc2);
        acc3 = fmaf(nr[n + 3], sWi[(n + 3) * kD + dcol], acc3);
      }
      for (; n < nact; ++n) acc0 = fmaf(nr[n], sWi[n * kD + dcol], acc0);
      sV[w * kD + dcol] = (acc0 + acc1) + (acc2 + acc3);
    }
  }
  __syncthreads();
  STAMP(2);

  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (wv < fa) {
    const int f = f0 + wv;
    const float* vw = sV + (wv * stride) * kD;       // U = rows of this frame's window
    const float ve0 = sV[wc * kD + L], ve1 = sV[(wc + 1) * kD + L];   // Ve[:, d = L]
    const bool kq = q < 2;                           // k = 4q + ks < 8

    // X0 = Wii @ U   (train.py:180): k = 4ks + q over the 8 window rows
    f32x4 x0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      x0 = mfma4(sm[SM_WII + L * kT + 4 * ks + q], vw[(4 * ks + q) * kD + L], x0);
    // E = Wv[:, :16] @ X0 (+ Wv[:, 16:18] @ Ve + bv)  (g2k_lstm_mcr.py:105,112)
    float wv16[4];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) wv16[ks] = L < kT ? sm[SM_WV + L * (kD + 2) + 4 * q + ks] : 0.f;
    f32x4 eN = {0.f, 0.f, 0.f, 0.f}, eT = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      eN = mfma4(wv16[ks], x0[ks], eN);      // E[4q+i][L]
      eT = mfma4(x0[ks], wv16[ks], eT);      // E[L][4q+i]
    }
    const float bvL = sm[SM_BV + L];
    // Rel = Ve * Ve (train.py:194-195), Rm = Wr @ Rel (g2k_lstm_mcr.py:106)
    float em[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 4 * q + i;
      if (kq) {
        eN[i] = (eN[i] + fmaf(sm[SM_WV + t * (kD + 2) + kD], ve0,
                              sm[SM_WV + t * (kD + 2) + kD + 1] * ve1)) + bvL;
        const float rm = fmaf(sm[SM_WR + 2 * t], ve0 * ve0, sm[SM_WR + 2 * t + 1] * (ve1 * ve1));
        em[i] = eN[i] * rm;
      } else {
        em[i] = 0.f;
      }
    }
    if (L < kT) {
      const float w16 = sm[SM_WV + L * (kD + 2) + kD], w17 = sm[SM_WV + L * (kD + 2) + kD + 1];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = 4 * q + i;
        eT[i] = (eT[i] + fmaf(w16, sV[wc * kD + d], w17 * sV[(wc + 1) * kD + d])) +
                sm[SM_BV + d];
      }
    }
    // A = g @ (E * Rm)  (g2k_lstm_mcr.py:105-106); cost = E @ g (:112-113)
    f32x4 aA = {0.f, 0.f, 0.f, 0.f}, cC = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float gA = kq ? sm[SM_G + L * kT + 4 * q + ks] : 0.f;            // g[r = L][t]
      const float gB = L < kT ? sm[SM_G + (4 * q + ks) * kT + L] : 0.f;      // g[d][t2 = L]
      aA = mfma4(gA, em[ks], aA);      // A[4q+i][L]
      cC = mfma4(eT[ks], gB, cC);      // cost[4q+i][L]
    }
    if (a.A_out) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a.A_out[(((size_t)s * F + f) * kD + 4 * q + i) * kD + L] = aA[i];
    }
    if (a.cost_out && kq && L < kT) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a.cost_out[(((size_t)s * F + f) * kT + 4 * q + i) * kT + L] = cC[i];
    }
    // As = softmax(exp(A) / cumsum(exp(A), axis 0), axis -1)  (train.py:240)
    // column L, rows 4q+i: running (max, sum exp) down the rows, exclusive
    // prefix over the four lane groups, then a 16-lane row softmax.
    {
      float m_i[4], s_i[4];
      float m = -INFINITY, sacc = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lse_combine(m, sacc, aA[i], 1.0f);
        m_i[i] = m; s_i[i] = sacc;
      }
      float mp = -INFINITY, sp = 0.f;
#pragma unroll
      for (int g = 0; g < 3; ++g) {
        const float mg = __shfl(m, L + 16 * g, 64);
        const float sg = __shfl(sacc, L + 16 * g, 64);
        if (g < q) lse_combine(mp, sp, mg, sg);
      }
      float ex[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float mr = m_i[i], sr = s_i[i];
        if (q > 0) lse_combine(mr, sr, mp, sp);
        const float R = __expf(aA[i] - mr) * rcp(sr);     // in (0, 1]
        ex[i] = __expf(R);
      }
      float* as = a.ws_as + ((size_t)s * F + f) * kD * kD;
#pragma unroll
      for (int i = 0; i < 4; ++i) as[(4 * q + i) * kD + L] = ex[i] * rcp(row16_sum(ex[i]));
    }
    // M^T = cost^T @ Wc^T for the x rows (jt 0) and y rows (jt 1) of temp_path
    f32x4 mT0 = {0.f, 0.f, 0.f, 0.f}, mT1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bool ok = kq && L < kL;
      const float wc0 = ok ? sm[SM_WC + L * kT + 4 * q + ks] : 0.f;
      const float wc1 = ok ? sm[SM_WC + (kL + L) * kT + 4 * q + ks] : 0.f;
      mT0 = mfma4(cC[ks], wc0, mT0);   // M[L][4q+i]       (x rows)
      mT1 = mfma4(cC[ks], wc1, mT1);   // M[12+L][4q+i]    (y rows)
    }
    // Y^T = Wo^T @ M^T per 16 pedestrians; pred_path_band = reshape(Y, (2,12,N))
    float* ys = smem + lay.o_y + wv * kD * kL2;
    const uint8_t* pm = a.ped_mask ? a.ped_mask + (size_t)s * Nmax : nullptr;
    const int pp = lane >> 2, u = lane & 3;             // error lanes: pedestrian, quarter
    const float* tgt_f = a.targets + ((size_t)s * F + f) * Nmax * kL2;
    float* pr = a.pred + ((size_t)s * F + f) * kL2 * Nmax;
    const int ntiles = (Nmax + 15) / 16;
    // targets of tiles t and t+1 are in flight while tile t is computed
    float2 tgB[3];
    auto load_tg = [&](int t, float2 (&tg)[3]) {
      const int ne = 16 * t + pp;
      const int nc = ne < Nmax ? ne : 0;
      const float2* tp = reinterpret_cast<const float2*>(tgt_f + (size_t)nc * kL2) + 3 * u;
      tg[0] = tp[0]; tg[1] = tp[1]; tg[2] = tp[2];
    };
    auto tile = [&](int t, const float2 (&tg)[3]) {
      const int n0 = 16 * t;
      const int ne = n0 + pp;
      const bool has_t = ne < nact && (pm ? pm[ne] != 0 : true);
      f32x4 y0 = {0.f, 0.f, 0.f, 0.f}, y1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int n = n0 + L;
        const float wo = (kq && n < nact) ? sWo[(4 * q + ks) * Nmax + n] : 0.f;
        y0 = mfma4(wo, mT0[ks], y0);   // Y[L][n0 + 4q + i]
        y1 = mfma4(wo, mT1[ks], y1);   // Y[12 + L][n0 + 4q + i]
      }
      if (L < kL) {
        const int nb = n0 + 4 * q;
        if (nb + 3 < Nmax && ((Nmax & 3) == 0)) {
          *reinterpret_cast<float4*>(pr + L * Nmax + nb) = make_float4(y0[0], y0[1], y0[2], y0[3]);
          *reinterpret_cast<float4*>(pr + (kL + L) * Nmax + nb) = make_float4(y1[0], y1[1], y1[2], y1[3]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (nb + i < Nmax) { pr[L * Nmax + nb + i] = y0[i]; pr[(kL + L) * Nmax + nb + i] = y1[i]; }
        }
        // transpose to [16 peds][12 steps][2] for the error lanes
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<float2*>(ys + (4 * q + i) * kL2 + 2 * L) = make_float2(y0[i], y1[i]);
      }
      __builtin_amdgcn_wave_barrier();
      // a9 errors (train.py:640-656): 4 lanes per pedestrian, 3 steps each
      float ea = 0.f, eb = 0.f, ec = 0.f, el2 = 0.f, fx = 0.f, fy = 0.f;
      const float2* yp = reinterpret_cast<const float2*>(ys + pp * kL2) + 3 * u;
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const float2 yv = yp[k];
        const float dx = yv.x - tg[k].x, dy = yv.y - tg[k].y;
        ea = fmaf(dx, dx, ea);
        eb = fmaf(dx, dy, eb);
        ec = fmaf(dy, dy, ec);
        el2 += sqrtf(fmaf(dx, dx, dy * dy));
        fx = dx; fy = dy;
      }
      __builtin_amdgcn_wave_barrier();
      // quad sums; the fde vector (step 11) lives in quarter 3
      ea += dpp<0xB1>(ea); ea += dpp<0x4E>(ea);
      eb += dpp<0xB1>(eb); eb += dpp<0x4E>(eb);
      ec += dpp<0xB1>(ec); ec += dpp<0x4E>(ec);
      el2 += dpp<0xB1>(el2); el2 += dpp<0x4E>(el2);
      fx = dpp<0xFF>(fx);   // quad_perm [3,3,3,3]
      fy = dpp<0xFF>(fy);
      if (has_t && u == 0) {
        const float hm = 0.5f * (ea - ec);
        const float lam = 0.5f * (ea + ec) + sqrtf(fmaf(hm, hm, eb * eb));
        const float fsq = fmaf(fx, fx, fy * fy);
        acc[0] += sqrtf(fmaxf(lam, 0.f)) * (1.0f / 12.0f);
        acc[1] += 1.0f;
        acc[2] += fsq;
        acc[3] += el2 * (1.0f / 12.0f);
        acc[4] += sqrtf(fsq);
      }
    };
    load_tg(1 < ntiles ? 1 : 0, tgB);
    for (int t = 0; t < ntiles; t += 2) {
      tile(t, tgA);
      if (t + 2 < ntiles) load_tg(t + 2, tgA);
      if (t + 1 < ntiles) {
        tile(t + 1, tgB);
        if (t + 3 < ntiles) load_tg(t + 3, tgB);
      }
    }
  }
  // ---- ADE/FDE partial sums of this chunk: fixed order, no atomics --------
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const float v = wave_sum(acc[k]);
    if (lane == 0) sMet[wv * 8 + k] = v;
  }
  __syncthreads();
  if (tid < 8) part[tid] = tid < 5 ? (sMet[tid] + sMet[8 + tid]) + (sMet[16 + tid] + sMet[24 + tid]) : 0.f;
  STAMP(6);
}

// ---------------------------------------------------------------------------
// Kernel 2: frame-sequential recurrence, one workgroup per scene.
// raw_attn = 0: `att` holds As (written by g2k_frames_kernel);
// raw_attn = 1: `att` holds A and the kernel applies train.py:240 itself.
// ---------------------------------------------------------------------------
struct RecurArgs {
  const float* att;      // [S, F, 16, 16]
  const float* h_in;
  float* h_out;
  const int32_t* n_frames;
  const float* ws_part;  // [S, nchunk, 8] or NULL
  float* metrics;        // [S, 8] or NULL
  int F, H, nchunk, raw_attn;
};

template <int TPW, int NW>
__global__ void __launch_bounds__(64 * NW) g2k_recur_kernel(RecurArgs a) {
  constexpr int kRT = 64 * NW;               // threads
  constexpr int kRB = 16 * NW;               // floats per row-partial buffer
  __shared__ __attribute__((aligned(16))) float sAs[kRecurChunk * kD * kD];
  __shared__ __attribute__((aligned(16))) float sRed[4 * kRB];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wv = wave_id(), q = lane >> 4, j = lane & 15;
  const int F = a.F, H = a.H;
  const int nf = a.n_frames ? clampi(a.n_frames[s], 0, F) : F;
  STAMP(10);
  // first As chunk, h and the metric partials all in flight together
  const int cnt0 = nf < kRecurChunk ? nf : kRecurChunk;
  if (nf > 0) dma_copy_n<kRT>(a.att + (size_t)s * F * kD * kD, sAs, cnt0 * (kD * kD / 4), wv, lane);
  Recur<TPW, NW> rec;
  rec.load(a.h_in + (size_t)s * kD * H, H, wv, q, j);
  if (a.metrics && tid < 8) {
    float v = 0.f;
    if (tid < 5) {
      const float* p = a.ws_part + (size_t)s * a.nchunk * 8 + tid;
      for (int c = 0; c < a.nchunk; ++c) v += p[c * 8];
    } else if (tid == 5) {
      v = (float)nf;
    }
    a.metrics[(size_t)s * 8 + tid] = v;
  }
  // sRed: three row-partial buffers rotated per frame + one for the row max
  const float* last = nullptr;
  if (nf > 0) {
    rec.init_max(sRed + 3 * kRB, wv, q, j);
    __syncthreads();
    rec.init_exp(sRed, sRed + 3 * kRB, wv, q, j);   // published by the chunk barrier below
    int cur = 0;
    for (int fb = 0; fb < nf; fb += kRecurChunk) {
      const int cnt = (nf - fb) < kRecurChunk ? (nf - fb) : kRecurChunk;
      if (fb > 0) dma_copy_n<kRT>(a.att + ((size_t)s * F + fb) * kD * kD, sAs, cnt * (kD * kD / 4), wv, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (a.raw_attn) {
        for (int task = tid; task < cnt * kD; task += kRT)
          attn_column_pass(sAs + (task >> 4) * kD * kD, task & 15);
        __syncthreads();
        for (int task = tid; task < cnt * kD; task += kRT)
          attn_row_pass(sAs + (task >> 4) * kD * kD, task & 15, nullptr);
        __syncthreads();
      }
      STAMP(11);
      for (int fl = 0; fl < cnt; ++fl) {
        const float4 b = *reinterpret_cast<const float4*>(sAs + fl * kD * kD + j * kD + 4 * q);
        const int nxt = cur == 2 ? 0 : cur + 1;
        rec.step(b, sRed + cur * kRB, sRed + nxt * kRB, wv, q, j);
        cur = nxt;
      }
      last = sRed + cur * kRB;
      __syncthreads();   // all waves done with sAs before the next DMA
    }
  }
  STAMP(12);
  rec.store(a.h_out + (size_t)s * kD * H, H, wv, q, j, last);
}

// ---------------------------------------------------------------------------
// Fused step (the default): g2k_scene_kernel, one workgroup per scene,
// wave-specialised.  Waves 0..3 (one per SIMD) run the frame-sequential
// recurrence (Recur::step_seq); waves 4..4+NP-1 are producers that run the
// frame-parallel body (frame_head + pred_tile below, frames pw, pw+NP, ...)
// and hand each frame's As tile to the recurrence through an LDS ring with a
// per-slot flag.  The two roles never share a barrier inside a chunk of
// frames, so the recurrence's latency chain runs while the producers stream
// predictions, targets and errors — and As never leaves the CU.
// Frames are processed in chunks of lay.fc (<= 32, LDS permitting); the
// workgroup barriers only at chunk boundaries.
// ---------------------------------------------------------------------------
constexpr int kSceneChunk = 32;
// scene kernel options (StepArgs::opts; G2K_SCENE_OPTS overrides the default)
constexpr int kOptRecHeads = 1;    // the recurrence waves head each chunk's first kRecW frames
constexpr int kOptValuTiles = 2;   // prediction tiles on the VALU (else MFMA)
constexpr int kModeDma16 = 4;      // 16-byte LDS-DMA staging (StepArgs::dma16)
// Defaults off: at eth_hotel_synth the recurrence-wave heads cost +1.3 us per
// step (they take ~4.5k cycles beside the staging tiles and delay the
// second barrier) and the VALU tiles +0.2 us (gpurun_out d30).
constexpr int kSceneOptsDefault = 0;
// A scene kernel is compiled per MODE (options | kModeDma16) so that each
// instantiation holds only the code it runs: every workgroup fetches its
// code cold at launch, and measured step time grows with the kernel's code
// bytes (~1.2 us per 8 KB at S = 256).
constexpr int kRecW = 4;
// scene-kernel small block: the split path's offsets plus weight-derived
// matrices (DESIGN.md "frame head"): K1 = [Wv16 @ Wii | Wv16.. | Wv17.. | 1 | 0]
// ([8][12]), K2 = Wc @ K1 ([24][12]).  G stays unscaled (lambda applied at use).
constexpr int SM_K1 = 640;
constexpr int SM_K2 = 752;
constexpr int kSceneSmall = 1088;
constexpr int kKA = 12;        // augmented contraction length (8 window rows + Ve0, Ve1, bv, 0)

struct SceneLayout {
  int fc, wcmax, pp;   // frames per chunk, window rows per chunk, pos row pitch (floats)
  int o_wi, o_wo, o_vis, o_v, o_small, o_y, o_met, o_ring, o_mring, o_flag, o_mflag, o_red, o_pos, o_vg;
  int total;   // floats
};

__host__ __device__ inline SceneLayout scene_layout_fc(int Nmax, int stride, int fc, int NP) {
  SceneLayout s;
  s.fc = fc;
  s.wcmax = (fc - 1) * stride + kT;
  s.pp = 2 * Nmax + 4;                        // padded rows: lanes reading across rows spread banks
  int o = 0;
  s.o_wi = o;    o += rup4(Nmax * kD);
  s.o_wo = o;    o += rup4(kT * Nmax);
  s.o_vis = o;   o += rup4(2 * Nmax);                  // vislet rows
  s.o_v = o;     o += rup4((s.wcmax + 2) * kD);        // V rows: window, Ve0, Ve1
  s.o_small = o; o += kSceneSmall;
  s.o_y = o;     o += NP * kD * kL2;                  // MFMA tiles' transpose scratch
  s.o_met = o;   o += NP * 8;
  s.o_ring = o;  o += fc * kD * kD;
  s.o_mring = o; o += fc * kL2 * kT;                  // M = Wc @ cost per frame [24][8]
  s.o_flag = o;  o += rup4(fc);                      // As ring flags (recurrence polls)
  s.o_mflag = o; o += rup4(fc);                      // M ring flags (prediction tiles poll)
  s.o_red = o;   o += 4 * 16 * kRecW;
  s.o_pos = o;   o += s.wcmax * s.pp;                  // raw position window (LDS-DMA)
  s.o_vg = o;    o += rup4((s.wcmax + 3) * kT);       // VG = V @ g: window, Ve0, Ve1, bv rows
  s.total = o;
  return s;
}

// frame head output: the x / y row tiles of M^T
// frame head output: the x / y row tiles of M^T
struct FrameHeadOut {
  f32x4 mT0, mT1;   // M[L][4q+i] (x rows), M[12+L][4q+i] (y rows)
};

// Partner lane's value across lane groups (q ^ 1 by permlane16, q ^ 2 by
// permlane32): of the pair a swap returns, one element is this lane's own
// value, the other the partner's.
__device__ __forceinline__ float partner16(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return a[0] == __float_as_uint(v) ? __uint_as_float(a[1]) : __uint_as_float(a[0]);
}
__device__ __forceinline__ float partner32(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return a[0] == __float_as_uint(v) ? __uint_as_float(a[1]) : __uint_as_float(a[0]);
}

// As = softmax(exp(A) / cumsum(exp(A), axis 0), axis -1)  (train.py:240) of
// one frame's A in the MFMA result layout (column L, rows 4q + i), written
// to as_dst [16][16].  The ratio exp(A_r) / sum_{k<=r} exp(A_k) is invariant
// to a per-column shift: with the column max M, e = exp(A - M) lies in (0, 1]
// and the prefix sums (in-lane, then across lane groups by permlane swaps)
// cannot overflow.  If a prefix sum underflows (the column's leading rows are
// ~87 below its max) the wave redoes the column with a running (max, sum)
// pair, which is exact for any finite A.  Then a 16-lane row softmax of
// values in (0, 1].
__device__ __forceinline__ void attn_weights(const f32x4 aA, float* as_dst, int L, int q) {
  float mx = fmaxf(fmaxf(aA[0], aA[1]), fmaxf(aA[2], aA[3]));
  mx = fmaxf(mx, partner16(mx));
  mx = fmaxf(mx, partner32(mx));
  float e[4], p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __expf(aA[i] - mx);
  p[0] = e[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) p[i] = p[i - 1] + e[i];
  const float t1 = partner16(p[3]), t2 = partner32(p[3]), t3 = partner32(t1);
  const float pre = ((q & 2) ? t2 + t3 : 0.f) + ((q & 1) ? t1 : 0.f);   // groups before q
  float R[4];
  bool bad = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float P = pre + p[i];
    bad |= !(P >= 1e-30f);
    R[i] = e[i] * rcp(P);
  }
  if (__builtin_amdgcn_ballot_w64(bad) != 0) {
    // running (max, sum exp) down the rows; exclusive prefix over the groups
    float m_i[4], s_i[4];
    float m = aA[0], sacc = 1.0f;
    m_i[0] = m; s_i[0] = sacc;
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      lse_combine(m, sacc, aA[i], 1.0f);
      m_i[i] = m; s_i[i] = sacc;
    }
    const float m1 = partner16(m), s1 = partner16(sacc);
    const float m2 = partner32(m), s2 = partner32(sacc);
    const float m3 = partner32(m1), s3 = partner32(s1);
    float pm = m2, ps = s2;
    lse_combine(pm, ps, m3, s3);
    float mp = -INFINITY, sp = 0.f;
    if (q & 2) { mp = pm; sp = ps; }
    if (q & 1) {
      if (q & 2) lse_combine(mp, sp, m1, s1);
      else { mp = m1; sp = s1; }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float mr = m_i[i], sr = s_i[i];
      if (q > 0) lse_combine(mr, sr, mp, sp);
      R[i] = __expf(aA[i] - mr) * rcp(sr);
    }
  }
  // stored as As * log2(e): the recurrence's A operand (Recur::body)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float ex = __expf(R[i]);
    as_dst[(4 * q + i) * kD + L] = ex * (rcp(row16_sum(ex)) * kLog2e);
  }
}

// frame head: the g2k_lstm_mcr forward of one frame up to M (models/
// g2k_lstm_mcr.py:99-124 with train.py:178-195), reassociated around the
// weight-derived K1 / K2 (computed once per workgroup in scene_stage):
//   E    = K1 @ Uaug      Uaug = [U (8 window rows of V); Ve0; Ve1; bv; 0]
//        = Wv[:, :16] @ (Wii @ U) + Wv[:, 16:18] @ Ve + bv          (:105, 112)
//   A    = g @ (E * Rm)                                             (:105-106)
//   cost = E @ g = K1 @ VGaug        (VGaug = Uaug @ g, rows of VG)  (:112-113)
//   M    = Wc @ cost = K2 @ VGaug                                   (:119)
// Contractions over the 12 augmented rows use k = 4 ks + q (3 k-steps);
// A contracts over t = 4q + ks (rows of E as the MFMA left them).
// As goes to `as_dst` (do_as); the x / y row tiles of M^T are returned
// (M[L][4q+i]).
__device__ __forceinline__ FrameHeadOut frame_head(const float* sm, const float* sV,
                                                   const float* sVG, int wrow0, int wcmax,
                                                   const float (&rm)[4], float lam, float* as_dst,
                                                   float* A_g, float* cost_g, int L, int q,
                                                   bool do_as) {
  float ka[3], ua[3], va[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int k = 4 * ks + q;
    ka[ks] = L < kT ? sm[SM_K1 + L * kKA + k] : 0.f;
    if (ks < 2) {
      ua[ks] = sV[(wrow0 + k) * kD + L];
      va[ks] = L < kT ? sVG[(wrow0 + k) * kT + L] : 0.f;
    } else {
      ua[ks] = q < 2 ? sV[(wcmax + q) * kD + L] : (q == 2 ? sm[SM_BV + L] : 0.f);
      va[ks] = L >= kT || q == 3 ? 0.f : sVG[(wcmax + q) * kT + L];   // Ve0, Ve1, bv rows
    }
  }
  f32x4 eN = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) eN = mfma4(ka[ks], ua[ks], eN);          // E[4q+i][L]
  FrameHeadOut o;
  o.mT0 = f32x4{0.f, 0.f, 0.f, 0.f};
  o.mT1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int k = 4 * ks + q;
    const float bx = L < kL ? sm[SM_K2 + L * kKA + k] : 0.f;
    const float by = L < kL ? sm[SM_K2 + (kL + L) * kKA + k] : 0.f;
    o.mT0 = mfma4(va[ks], bx, o.mT0);   // M[L][4q+i]       (x rows)
    o.mT1 = mfma4(va[ks], by, o.mT1);   // M[12+L][4q+i]    (y rows)
  }
  f32x4 aA = {0.f, 0.f, 0.f, 0.f};
  if (do_as || A_g) {
    float em[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) em[i] = eN[i] * rm[i];                    // rm = 0 for t >= 8
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const float gA = q < 2 ? lam * sm[SM_G + L * kT + 4 * q + ks] : 0.f;  // g[r = L][t]
      aA = mfma4(gA, em[ks], aA);                                        // A[4q+i][L]
    }
  }
  if (A_g) {
#pragma unroll
    for (int i = 0; i < 4; ++i) A_g[(4 * q + i) * kD + L] = aA[i];
  }
  if (cost_g) {
    f32x4 cC = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) cC = mfma4(ka[ks], va[ks], cC);      // cost[4q+i][L]
    if (q < 2 && L < kT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) cost_g[(4 * q + i) * kT + L] = cC[i];
    }
  }
  if (do_as) attn_weights(aA, as_dst, L, q);
  return o;
}

// One 16-pedestrian tile of one frame on the VALU (the matrix pipe is left
// to the recurrence waves, which share the SIMDs): Y[r][n] = sum_t M[r][t]
// Wo[t][n] (models/g2k_lstm_mcr.py:122; M = the frame's [24][8] from the M
// ring).  Lane (pp = lane >> 2, u = lane & 3) owns pedestrian n = 16 t + pp
// and prediction steps 3u .. 3u + 2 (x and y rows): it stores them and forms
// the a9 error terms of its steps; the four lanes of a pedestrian are summed
// by DPP quad exchanges.
__device__ __forceinline__ void pred_tile(const float* M, const float* sWo, float* pr,
                                          const float2 (&tg)[3], const uint8_t* pm, int Nmax,
                                          int nact, int t, int lane, float acc[5]) {
  const int pp = lane >> 2, u = lane & 3;
  const int n = 16 * t + pp;
  const int nc = n < Nmax ? n : Nmax - 1;
  const bool live = n < nact;
  const bool has_t = live && (pm ? pm[nc] != 0 : true);
  float wo[kT];
#pragma unroll
  for (int k = 0; k < kT; ++k) wo[k] = live ? sWo[k * Nmax + nc] : 0.f;
  float yx[3], yy[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float4* mx = reinterpret_cast<const float4*>(M + (3 * u + j) * kT);
    const float4* my = reinterpret_cast<const float4*>(M + (kL + 3 * u + j) * kT);
    const float4 x0 = mx[0], x1 = mx[1], y0 = my[0], y1 = my[1];
    float sx = x0.x * wo[0], sy = y0.x * wo[0];
    sx = fmaf(x0.y, wo[1], sx); sy = fmaf(y0.y, wo[1], sy);
    sx = fmaf(x0.z, wo[2], sx); sy = fmaf(y0.z, wo[2], sy);
    sx = fmaf(x0.w, wo[3], sx); sy = fmaf(y0.w, wo[3], sy);
    sx = fmaf(x1.x, wo[4], sx); sy = fmaf(y1.x, wo[4], sy);
    sx = fmaf(x1.y, wo[5], sx); sy = fmaf(y1.y, wo[5], sy);
    sx = fmaf(x1.z, wo[6], sx); sy = fmaf(y1.z, wo[6], sy);
    sx = fmaf(x1.w, wo[7], sx); sy = fmaf(y1.w, wo[7], sy);
    yx[j] = sx;
    yy[j] = sy;
  }
  if (n < Nmax) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      pr[(3 * u + j) * Nmax + n] = yx[j];
      pr[(kL + 3 * u + j) * Nmax + n] = yy[j];
    }
  }
  float ea = 0.f, eb = 0.f, ec = 0.f, el2 = 0.f, fx = 0.f, fy = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float dx = yx[k] - tg[k].x, dy = yy[k] - tg[k].y;
    ea = fmaf(dx, dx, ea);
    eb = fmaf(dx, dy, eb);
    ec = fmaf(dy, dy, ec);
    el2 += __builtin_amdgcn_sqrtf(fmaf(dx, dx, dy * dy));
    fx = dx; fy = dy;
  }
  ea += dpp<0xB1>(ea); ea += dpp<0x4E>(ea);
  eb += dpp<0xB1>(eb); eb += dpp<0x4E>(eb);
  ec += dpp<0xB1>(ec); ec += dpp<0x4E>(ec);
  el2 += dpp<0xB1>(el2); el2 += dpp<0x4E>(el2);
  fx = dpp<0xFF>(fx);   // quad_perm [3,3,3,3]: the fde vector lives in quarter 3
  fy = dpp<0xFF>(fy);
  if (has_t && u == 0) {
    const float hm = 0.5f * (ea - ec);
    const float lam = 0.5f * (ea + ec) + __builtin_amdgcn_sqrtf(fmaf(hm, hm, eb * eb));
    const float fsq = fmaf(fx, fx, fy * fy);
    acc[0] += __builtin_amdgcn_sqrtf(fmaxf(lam, 0.f)) * (1.0f / 12.0f);
    acc[1] += 1.0f;
    acc[2] += fsq;
    acc[3] += el2 * (1.0f / 12.0f);
    acc[4] += __builtin_amdgcn_sqrtf(fsq);
  }
}

// The same tile by MFMA (scene option kOptValuTiles off): Y^T = Wo^T @ M^T (M = this frame's
// [24][8] from the M ring), pred stores, a9 error terms (4 lanes per
// pedestrian) accumulated into acc.  The contraction over t (8) uses
// k = 4 ks + q, so two k-steps cover it without zero padding.
__device__ __forceinline__ void pred_tile_mfma(const float* M, const float* sWo, float* ys,
                                          float* pr, const float2 (&tg)[3], const uint8_t* pm,
                                          int Nmax, int nact, int t, int L, int q, int lane,
                                          float acc[5]) {
  const int pp = lane >> 2, u = lane & 3;
  const int n0 = 16 * t;
  const int ne = n0 + pp;
  const bool has_t = ne < nact && (pm ? pm[ne] != 0 : true);
  f32x4 y0 = {0.f, 0.f, 0.f, 0.f}, y1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int n = n0 + L, k = 4 * ks + q;
    const float wo = n < nact ? sWo[k * Nmax + n] : 0.f;
    const float bx = L < kL ? M[L * kT + k] : 0.f;
    const float by = L < kL ? M[(kL + L) * kT + k] : 0.f;
    y0 = mfma4(wo, bx, y0);   // Y[L][n0 + 4q + i]
    y1 = mfma4(wo, by, y1);   // Y[12 + L][n0 + 4q + i]
  }
  if (L < kL) {
    const int nb = n0 + 4 * q;
    if (nb + 3 < Nmax && ((Nmax & 3) == 0)) {
      *reinterpret_cast<float4*>(pr + L * Nmax + nb) = make_float4(y0[0], y0[1], y0[2], y0[3]);
      *reinterpret_cast<float4*>(pr + (kL + L) * Nmax + nb) = make_float4(y1[0], y1[1], y1[2], y1[3]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (nb + i < Nmax) { pr[L * Nmax + nb + i] = y0[i]; pr[(kL + L) * Nmax + nb + i] = y1[i]; }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<float2*>(ys + (4 * q + i) * kL2 + 2 * L) = make_float2(y0[i], y1[i]);
  }
  __builtin_amdgcn_wave_barrier();
  float ea = 0.f, eb = 0.f, ec = 0.f, el2 = 0.f, fx = 0.f, fy = 0.f;
  const float2* yp = reinterpret_cast<const float2*>(ys + pp * kL2) + 3 * u;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float2 yv = yp[k];
    const float dx = yv.x - tg[k].x, dy = yv.y - tg[k].y;
    ea = fmaf(dx, dx, ea);
    eb = fmaf(dx, dy, eb);
    ec = fmaf(dy, dy, ec);
    el2 += __builtin_amdgcn_sqrtf(fmaf(dx, dx, dy * dy));
    fx = dx; fy = dy;
  }
  __builtin_amdgcn_wave_barrier();
  ea += dpp<0xB1>(ea); ea += dpp<0x4E>(ea);
  eb += dpp<0xB1>(eb); eb += dpp<0x4E>(eb);
  ec += dpp<0xB1>(ec); ec += dpp<0x4E>(ec);
  el2 += dpp<0xB1>(el2); el2 += dpp<0x4E>(el2);
  fx = dpp<0xFF>(fx);   // quad_perm [3,3,3,3]: the fde vector lives in quarter 3
  fy = dpp<0xFF>(fy);
  if (has_t && u == 0) {
    const float hm = 0.5f * (ea - ec);
    const float lam = 0.5f * (ea + ec) + __builtin_amdgcn_sqrtf(fmaf(hm, hm, eb * eb));
    const float fsq = fmaf(fx, fx, fy * fy);
    acc[0] += __builtin_amdgcn_sqrtf(fmaxf(lam, 0.f)) * (1.0f / 12.0f);
    acc[1] += 1.0f;
    acc[2] += fsq;
    acc[3] += el2 * (1.0f / 12.0f);
    acc[4] += __builtin_amdgcn_sqrtf(fsq);
  }
}

// Per-workgroup context of the scene kernel (LDS carve-up, scene scalars).
struct SceneCtx {
  float *sWi, *sWo, *sVis, *sV, *sm, *sMet, *sRing, *sMring, *sRed, *sPos, *sVG, *sY;
  int* sFlag;     // As ring: global frame + 1 once the frame's As is in its slot
  int* sMflag;    // M ring: global frame + 1 once the frame's M is in its slot
  int* sTicket;   // producers' metrics ticket (after the recurrence sequence words)
  int s, tid, lane, wv, L, q, nact, nf, ntiles;
};

// LDS-DMA of a chunk's position window rows (train.py:76-79 window) into
// rows of pitch lay.pp: wave w issues rows w, w + waves, ...
template <int NT>
__device__ __forceinline__ void scene_pos_dma(const StepArgs& a, const SceneLayout& lay,
                                              const SceneCtx& c, int fb, int cnt) {
  const int Nmax = a.d.Nmax, stride = a.d.stride;
  const int wcc = (cnt - 1) * stride + kT;
  const float* src = a.pos + ((size_t)c.s * a.d.W + fb * stride) * Nmax * 2;
  const bool wide = (Nmax & 1) == 0 && (((uintptr_t)a.pos) & 15) == 0;
  for (int r = c.wv; r < wcc; r += NT / 64) {
    const float* g = src + (size_t)r * Nmax * 2;
    float* d = c.sPos + r * lay.pp;
    if (wide) {
      for (int i = 0; i < Nmax / 2; i += 64)
        if (i + c.lane < Nmax / 2) dma16(g + 4 * (i + c.lane), d + 4 * i);
    } else {
      for (int i = 0; i < 2 * Nmax; i += 64)
        if (i + c.lane < 2 * Nmax)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + i + c.lane),
                                           (__attribute__((address_space(3))) void*)(d + i), 4, 0, 0);
    }
  }
}

// The scene's inputs by 16-byte LDS-DMA, in few full-width instructions
// (every LDS-DMA instruction costs the CU's vector-memory path about the
// same whatever its width, so the prologue issues ~18 of them instead of
// ~65 narrow ones).  Instruction k of the workgroup (wave k % waves) covers
// 64 consecutive 16-B slots of one segment; the LDS image of each segment is
// contiguous in slot order, so the LDS destination is the instruction's
// base + 16 * lane as LDS-DMA requires.  Segment 0 is the position window
// with rows padded to R + 1 slots (R = Nmax / 2; the pad slot re-reads the
// row's first slot); with `weights` the weight / per-scene blocks follow.
// Requires StepArgs::dma16 (checked on the host).
template <int NT>
__device__ __forceinline__ void scene_dma16(const StepArgs& a, const SceneLayout& lay,
                                            const SceneCtx& c, int fb, int cnt, bool weights) {
  const int Nmax = a.d.Nmax, R = Nmax >> 1, stride = a.d.stride;
  const int wcc = (cnt - 1) * stride + kT;
  const int npos = wcc * (R + 1);
  const int ipos = (npos + 63) >> 6;
  const float* psrc = a.pos + ((size_t)c.s * a.d.W + (size_t)fb * stride) * Nmax * 2;
  constexpr int kSeg = 9;
  const float* src[kSeg] = {a.w.Wi, a.w.Wo, a.w.Wii, a.w.Wv, a.w.bv, a.w.Wr, a.w.Wc,
                            a.G + (size_t)c.s * kD * kT, a.vislet + (size_t)c.s * 2 * Nmax};
  float* dst[kSeg] = {c.sWi, c.sWo, c.sm + SM_WII, c.sm + SM_WV, c.sm + SM_BV, c.sm + SM_WR,
                      c.sm + SM_WC, c.sm + SM_G, c.sVis};
  const int n16[kSeg] = {4 * Nmax, 2 * Nmax, kD * kT / 4, kT * (kD + 2) / 4, kD / 4, kT * 2 / 4,
                         kL2 * kT / 4, kD * kT / 4, R};
  int ninst = ipos;
  if (weights) {
#pragma unroll
    for (int i = 0; i < kSeg; ++i) ninst += (n16[i] + 63) >> 6;
  }
  for (int k = c.wv; k < ninst; k += NT / 64) {
    if (k < ipos) {
      const int t = 64 * k + c.lane;
      if (t < npos) {
        const int row = t / (R + 1);
        int col = t - row * (R + 1);
        col = col == R ? 0 : col;
        dma16(psrc + (size_t)row * 2 * Nmax + 4 * col, c.sPos + 256 * k);
      }
    } else {
      int j = k - ipos;
#pragma unroll
      for (int i = 0; i < kSeg; ++i) {
        const int ni = (n16[i] + 63) >> 6;
        if (j >= 0 && j < ni) {
          const int t = 64 * j + c.lane;
          if (t < n16[i]) dma16(src[i] + 4 * t, dst[i] + 256 * j);
        }
        j -= ni;
      }
    }
  }
}

// One 16-row tile of the chunk's embedding rows, by MFMA (train.py:76-79,
// 167-195): local rows r = w0 + L are the window rows (r < wcc: norms
// ||pos||, formed here from the LDS window), the two vislet rows and a bv
// pseudo-row (VG only).  V^T = Wi^T @ N^T over n (k = 4 ks + q), then
// VG^T = (lambda G)^T @ V^T over d with V^T straight from the registers.
// Lane (L, q) ends with V[r][4q..4q+3] and VG[r][4q..4q+3] (q < 2).
__device__ __forceinline__ void scene_vtile(const StepArgs& a, const SceneLayout& lay,
                                            const SceneCtx& c, int w0, int wcc) {
  // branch-free: every lane loads at clamped addresses and selects, so the
  // LDS reads of several k-steps are in flight together
  const int Nmax = a.d.Nmax, L = c.L, q = c.q, nact = c.nact;
  const int r = w0 + L;
  const bool win = r < wcc, vis = r >= wcc && r < wcc + 2, bvrow = r == wcc + 2;
  const float* prow = c.sPos + (win ? r : 0) * lay.pp;
  const float* vrow = c.sVis + (vis ? r - wcc : 0) * Nmax;
  struct Raw { float wi, px, py, v; };
  auto load = [&](int ks) {
    const int n = 4 * ks + q;
    const int nc = n < Nmax ? n : Nmax - 1;
    const float2 p = *reinterpret_cast<const float2*>(prow + 2 * nc);
    return Raw{c.sWi[nc * kD + L], p.x, p.y, vrow[nc]};           // Wi[n][d = L], pos, vislet
  };
  auto value = [&](int ks, const Raw& w) {                         // N[w0 + L][n]
    const int n = 4 * ks + q;
    const float nrm = __builtin_amdgcn_sqrtf(fmaf(w.px, w.px, w.py * w.py));
    return n < nact ? (win ? nrm : (vis ? w.v : 0.f)) : 0.f;
  };
  const int nks = (Nmax + 3) / 4;
  f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
  SSTAMP(114, c.lane == 0 && w0 == 0);
  int ks = 0;
  for (; ks + 4 <= nks; ks += 4) {
    Raw r0 = load(ks), r1 = load(ks + 1), r2 = load(ks + 2), r3 = load(ks + 3);
    // keep all twelve loads unconditional and in flight together
    asm volatile("" : "+v"(r0.wi), "+v"(r0.px), "+v"(r0.py), "+v"(r0.v), "+v"(r1.wi), "+v"(r1.px),
                 "+v"(r1.py), "+v"(r1.v), "+v"(r2.wi), "+v"(r2.px), "+v"(r2.py), "+v"(r2.v),
                 "+v"(r3.wi), "+v"(r3.px), "+v"(r3.py), "+v"(r3.v));
    v0 = mfma4(r0.wi, value(ks, r0), v0);                          // V[w0 + L][4q + i]
    v1 = mfma4(r1.wi, value(ks + 1, r1), v1);
    v0 = mfma4(r2.wi, value(ks + 2, r2), v0);
    v1 = mfma4(r3.wi, value(ks + 3, r3), v1);
  }
  for (; ks < nks; ++ks) {
    Raw r0 = load(ks);
    asm volatile("" : "+v"(r0.wi), "+v"(r0.px), "+v"(r0.py), "+v"(r0.v));
    v0 = mfma4(r0.wi, value(ks, r0), v0);
  }
  f32x4 vt;
#pragma unroll
  for (int i = 0; i < 4; ++i) vt[i] = v0[i] + v1[i];
  SSTAMP(115, c.lane == 0 && w0 == 0);
  f32x4 vg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks2 = 0; ks2 < 4; ++ks2) {
    const float gl = c.sm[SM_G + (4 * q + ks2) * kT + (L & 7)];
    const float ga = L < kT ? a.lambda * gl : 0.f;                          // g[d][t2 = L]
    const float bvv = c.sm[SM_BV + 4 * q + ks2];
    vg = mfma4(ga, bvrow ? bvv : vt[ks2], vg);                             // VG[w0 + L][4q + i]
  }
  const int row = win ? r : lay.wcmax + (r - wcc);               // storage row
  if (win || vis)
    *reinterpret_cast<float4*>(c.sV + row * kD + 4 * q) = make_float4(vt[0], vt[1], vt[2], vt[3]);
  if ((win || vis || bvrow) && q < 2)
    *reinterpret_cast<float4*>(c.sVG + row * kT + 4 * q) = make_float4(vg[0], vg[1], vg[2], vg[3]);
}

// K1 = [Wv[:, :16] @ Wii | Wv[:, 16] | Wv[:, 17] | 1 | 0] ([8][12]) and
// K2 = Wc @ K1 ([24][12]) by MFMA in one wave (weights only; see frame_head).
__device__ __forceinline__ void scene_kmats(const SceneCtx& c) {
  const int L = c.L, q = c.q, L7 = L & 7;
  const float* sm = c.sm;
  float av[4], bw[4];
  float wv16[4], wv17[4], wc0[4], wc1[4];
  const int q1 = q & 1;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int d = 4 * q + ks;
    av[ks] = sm[SM_WV + L7 * (kD + 2) + d];                      // Wv[t = L][d]
    bw[ks] = sm[SM_WII + d * kT + L7];                           // Wii[d][k = L]
    const int t = 4 * q1 + ks;
    wv16[ks] = sm[SM_WV + t * (kD + 2) + kD];
    wv17[ks] = sm[SM_WV + t * (kD + 2) + kD + 1];
    wc0[ks] = sm[SM_WC + L * kT + 4 * q1 + ks];                 // Wc rows 0..15
    wc1[ks] = sm[SM_WC + (16 + L7) * kT + 4 * q1 + ks];        // Wc rows 16..23
  }
  asm volatile("" : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]), "+v"(bw[0]), "+v"(bw[1]),
               "+v"(bw[2]), "+v"(bw[3]));
  asm volatile("" : "+v"(wc0[0]), "+v"(wc0[1]), "+v"(wc0[2]), "+v"(wc0[3]), "+v"(wc1[0]),
               "+v"(wc1[1]), "+v"(wc1[2]), "+v"(wc1[3]));
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    av[ks] = L < kT ? av[ks] : 0.f;
    bw[ks] = L < kT ? bw[ks] : 0.f;
    wc0[ks] = q < 2 ? wc0[ks] : 0.f;
    wc1[ks] = (q < 2 && L < kL2 - 16) ? wc1[ks] : 0.f;
  }
  f32x4 k1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) k1 = mfma4(av[ks], bw[ks], k1);   // K1[4q + i][L]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = k1[i];
    v = L == 8 ? wv16[i] : L == 9 ? wv17[i] : L == 10 ? 1.f : L == 11 ? 0.f : v;
    k1[i] = (q < 2 && L < kKA) ? v : 0.f;
  }
  f32x4 ka = {0.f, 0.f, 0.f, 0.f}, kb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    ka = mfma4(wc0[ks], k1[ks], ka);                               // K2[4q + i][L]
    kb = mfma4(wc1[ks], k1[ks], kb);                               // K2[16 + 4q + i][L]
  }
  if (L < kKA) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 4 * q + i;
      if (q < 2) c.sm[SM_K1 + t * kKA + L] = k1[i];
      c.sm[SM_K2 + t * kKA + L] = ka[i];
      if (16 + t < kL2) c.sm[SM_K2 + (16 + t) * kKA + L] = kb[i];
    }
  }
}

// The first kRecW frame heads of a chunk on the recurrence waves (wave w:
// chunk frame w), between the staging barriers: they read only the LDS
// window and the weights (not the staging tiles' V / VG or K1 / K2), so they
// run beside the producers' staging and As_0 is in the ring when the
// recurrence starts instead of one producer head later.  Only As
// (train.py:240) is formed here; these frames' M and optional A / cost
// outputs stay with the producers (frame_head with do_as = false).
// v_mfma_f32_16x16x4_f32 chain (lane (L, q), register i = row 4q + i):
//   K1^T = Wii^T @ Wv[:, :16]^T        K1[t = L][4q + i]: the A operand of E
//   Vaug = Naug @ Wi                   rows 0..7 the frame's window norms
//                                      (train.py:76-85), 8, 9 the vislet rows
//                                      (Ve, train.py:182-183)
//   E    = [K1 | Wv16 | Wv17] @ Vaug + bv              (g2k_lstm_mcr.py:105)
//   A    = (lambda G) @ (E * Rm),  Rm = Wr @ (Ve * Ve)  (:105-106)
__device__ __forceinline__ void scene_rec_head(const StepArgs& a, const SceneLayout& lay,
                                               const SceneCtx& c, int fb, int fl) {
  const int Nmax = a.d.Nmax, L = c.L, q = c.q, L7 = L & 7, nact = c.nact;
  const float* sm = c.sm;
  float aw[4], bw[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int d = 4 * q + ks;
    aw[ks] = L < kT ? sm[SM_WII + d * kT + L7] : 0.f;          // Wii[d][m = L]
    bw[ks] = L < kT ? sm[SM_WV + L7 * (kD + 2) + d] : 0.f;     // Wv[t = L][d]
  }
  f32x4 k1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) k1 = mfma4(aw[ks], bw[ks], k1);   // K1[L][4q + i]
  // Vaug: A operand Naug[r = L][n], B operand Wi[n][d = L], n = 4 ks + q
  const bool win = L < kT, vis = L == kT || L == kT + 1;
  const float* prow = c.sPos + (fl * a.d.stride + L7) * lay.pp;
  const float* vrow = c.sVis + (L == kT + 1 ? Nmax : 0);
  auto nload = [&](int ks, float& wi, float2& p, float& v) {
    const int n = 4 * ks + q;
    const int nc = n < Nmax ? n : Nmax - 1;
    wi = c.sWi[nc * kD + L];
    p = *reinterpret_cast<const float2*>(prow + 2 * nc);
    v = vrow[nc];
  };
  auto nval = [&](int ks, const float2 p, float v) {
    const int n = 4 * ks + q;
    const float nrm = __builtin_amdgcn_sqrtf(fmaf(p.x, p.x, p.y * p.y));
    return n < nact ? (win ? nrm : (vis ? v : 0.f)) : 0.f;
  };
  const int nks = (Nmax + 3) / 4;
  f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
  int ks = 0;
  for (; ks + 2 <= nks; ks += 2) {
    float w0, w1, u0, u1;
    float2 p0, p1;
    nload(ks, w0, p0, u0);
    nload(ks + 1, w1, p1, u1);
    v0 = mfma4(nval(ks, p0, u0), w0, v0);
    v1 = mfma4(nval(ks + 1, p1, u1), w1, v1);
  }
  if (ks < nks) {
    float w0, u0;
    float2 p0;
    nload(ks, w0, p0, u0);
    v0 = mfma4(nval(ks, p0, u0), w0, v0);
  }
  f32x4 vt;
#pragma unroll
  for (int i = 0; i < 4; ++i) vt[i] = v0[i] + v1[i];            // Vaug[4q + i][L]
  f32x4 eN = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float ak = q < 2 ? k1[k] : ((q == 2 && k < 2) ? sm[SM_WV + L7 * (kD + 2) + kD + k] : 0.f);
    eN = mfma4(L < kT ? ak : 0.f, vt[k], eN);                    // E[4q + i][L] - bv[L]
  }
  // Ve rows live in lane group q = 2 (registers 0, 1): fetch column L's
  const float ve0 = __int_as_float(__builtin_amdgcn_ds_bpermute((L + 32) << 2, __float_as_int(vt[0])));
  const float ve1 = __int_as_float(__builtin_amdgcn_ds_bpermute((L + 32) << 2, __float_as_int(vt[1])));
  const float bvl = sm[SM_BV + L];
  float em[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = 4 * q + i;
    const float rm = q < 2 ? fmaf(sm[SM_WR + 2 * t], ve0 * ve0, sm[SM_WR + 2 * t + 1] * (ve1 * ve1)) : 0.f;
    em[i] = (eN[i] + bvl) * rm;
  }
  f32x4 aA = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gA = q < 2 ? a.lambda * sm[SM_G + L * kT + 4 * q + k] : 0.f;   // g[r = L][t]
    aA = mfma4(gA, em[k], aA);                                              // A[4q + i][L]
  }
  attn_weights(aA, c.sRing + fl * kD * kD, L, q);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (c.lane == 0) lds_store_flag(c.sFlag + fl, fb + fl + 1);
}

// Chunk staging shared by both roles (every wave takes part).  The chunk's
// position window is in flight by LDS-DMA.  Wait, barrier; the producer
// waves compute the embedding-row tiles (scene_vtile) and, at the first
// chunk, K1 / K2 (scene_kmats) while `rec_init` runs on the recurrence
// waves (softmax(h) numerators, the first frame heads); barrier.
template <int NT, int NP, int VMC, typename RecInit>
__device__ __forceinline__ void scene_stage(const StepArgs& a, const SceneLayout& lay,
                                            const SceneCtx& c, int fb, int cnt, RecInit rec_init) {
  const int wcc = (cnt - 1) * a.d.stride + kT;
  // VMC = vector-memory ops this wave issued after the LDS-DMA that may stay
  // in flight (the recurrence's h loads at the first chunk)
  if (VMC > 0 && fb == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(VMC) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  SSTAMP(102, c.tid == 0 && fb == 0);
  __syncthreads();                                              // B1: window + weights landed
  SSTAMP(1, c.tid == 0 && fb == 0);
  if (c.wv >= kRecW) {
    const int ntile = (wcc + 3 + 15) / 16;
    const int ntask = ntile + (fb == 0 ? 1 : 0);
    for (int task = c.wv - kRecW; task < ntask; task += NP) {
      if (task < ntile) scene_vtile(a, lay, c, 16 * task, wcc);
      else scene_kmats(c);
      SSTAMP(105 + (task & 7), c.lane == 0 && fb == 0);
    }
  } else {
    rec_init();
    SSTAMP(113, c.tid == 0 && fb == 0);
  }
  __syncthreads();                                              // B2: V, VG, K1, K2
  SSTAMP(2, c.tid == 0 && fb == 0);
  SSTAMP(101, c.tid == 0 && fb == 0);
}

// Role 1: the recurrence (waves 0..3).
template <int TPW, int NP, int MODE>
__device__ __forceinline__ void scene_recurrence(const StepArgs& a, const SceneLayout& lay,
                                                 const SceneCtx& c) {
  constexpr int NT = 64 * (kRecW + NP);
  constexpr int kRB = 16 * kRecW;
  const int H = a.d.H;
  Recur<TPW, kRecW> rc;
  asm volatile("" ::: "memory");   // h loads after the prologue's LDS-DMA (counted vmcnt)
  rc.load(a.h_in + (size_t)c.s * kD * H, H, c.wv, c.q, c.L);
  asm volatile("" ::: "memory");
  int* seq = reinterpret_cast<int*>(c.sRed + 2 * kRB);   // 2 partial buffers, seq words, row max
  for (int fb = 0; fb < c.nf; fb += lay.fc) {
    const int cnt = (c.nf - fb) < lay.fc ? (c.nf - fb) : lay.fc;
    if (fb > 0) {
      if constexpr ((MODE & kModeDma16) != 0) scene_dma16<NT>(a, lay, c, fb, cnt, false);
      else scene_pos_dma<NT>(a, lay, c, fb, cnt);
    }
    scene_stage<NT, NP, TPW * 4>(a, lay, c, fb, cnt, [&] {
      // softmax(h) numerators (first chunk): row max exchange (seq 1), then
      // e and its row partials into buffer 0 (seq 2), no workgroup barrier;
      // the chunk's first kRecW frame heads in between (scene_rec_head)
      if (fb == 0) {
        rc.init_max(c.sRed + 3 * kRB, c.wv, c.q, c.L);
        asm volatile("" ::: "memory");
        if (c.lane == 0) lds_store_flag(seq + c.wv, 1);
      }
      if constexpr ((MODE & kOptRecHeads) != 0) {
        if (c.wv < cnt) scene_rec_head(a, lay, c, fb, c.wv);
      }
      SSTAMP(74 + c.wv, c.lane == 0 && fb == 0);
      if (fb == 0) {
        poll_seq(seq + (c.L & 3), 1);
        rc.init_exp(c.sRed, c.sRed + 3 * kRB, c.wv, c.q, c.L);
        asm volatile("" ::: "memory");
        if (c.lane == 0) lds_store_flag(seq + c.wv, 2);
      }
    });
    __builtin_amdgcn_s_setprio(2);
    const float* as_lane = c.sRing + c.L * kD + 4 * c.q;   // this lane's As row quad, frame 0 of the ring
    // one frame; (b, flq): this frame's prefetched As quad and flag, (bn,
    // fln): where the next frame's prefetch goes.  Unrolled by two with the
    // pairs swapped so that a prefetch never needs a register copy (a copy
    // at the loop edge waits for every outstanding LDS op, the publish too).
    auto frame = [&](int fl, float4& b, int& flq, float4& bn, int& fln) {
      const int g = fb + fl;                 // global frame index
      float4 z;
#ifndef G2K_DIAG_FEW_STAMPS
      SSTAMP(116 + c.wv, c.lane == 0 && g == 10);
#endif
      poll_red(seq + (c.L & 3), g + 2, c.sRed + (g & 1) * kRB + (c.L & 3) * 16 + 4 * c.q, z);
      if (__builtin_amdgcn_readfirstlane(flq) != g + 1) wait_as(c.sFlag + fl, g + 1, as_lane + fl * kD * kD, b);
#ifndef G2K_DIAG_FEW_STAMPS
      SSTAMP(120 + c.wv, c.lane == 0 && g == 10);
#endif
      const int fn = fl + 1 < cnt ? fl + 1 : fl;   // next frame's ring slot (itself at the end)
      rc.step_seq(b, z, c.sRed + ((g + 1) & 1) * kRB, seq, g + 3, c.wv, c.q, c.L, c.sFlag + fn,
                  as_lane + fn * kD * kD, fln, bn);
#ifndef G2K_DIAG_FEW_STAMPS
      SSTAMP(124 + c.wv, c.lane == 0 && g == 10);
      SSTAMP(40 + ((fb + fl) & 31), c.tid == 0);
#else
      SSTAMP(40 + ((fb + fl) & 31), c.tid == 0 && (g == 0 || g == 10 || g + 1 == c.nf));
#endif
    };
    float4 b0, b1;
    int f0 = read_as(c.sFlag, as_lane, b0), f1 = 0;
    for (int fl = 0; fl < cnt; fl += 2) {
      frame(fl, b0, f0, b1, f1);
      if (fl + 1 < cnt) frame(fl + 1, b1, f1, b0, f0);
    }
#ifdef G2K_DIAG_RECUR_REPEAT
    // diagnostic build only: 1000 more recurrence frames on frame 0's As
    // after the real ones (the producers are done by then): the steady-state
    // cost of one frame inside this kernel, stamps 72 / 73
    if (fb + lay.fc >= c.nf) {
      SSTAMP(72, c.tid == 0);
      float4 ba, bb;
      int fa = read_as(c.sFlag, as_lane, ba), fbb = 0;
      int sl = 0;   // ring slot cycling through the chunk's real As tiles
      for (int it = 0; it < 1000; it += 2) {
        const int g0 = c.nf + it, g1 = g0 + 1;
        float4 z;
        sl = sl + 1 < cnt ? sl + 1 : 0;
        poll_red(seq + (c.L & 3), g0 + 2, c.sRed + (g0 & 1) * kRB + (c.L & 3) * 16 + 4 * c.q, z);
        rc.step_seq(ba, z, c.sRed + ((g0 + 1) & 1) * kRB, seq, g0 + 3, c.wv, c.q, c.L, c.sFlag + sl,
                    as_lane + sl * kD * kD, fbb, bb);
        sl = sl + 1 < cnt ? sl + 1 : 0;
        poll_red(seq + (c.L & 3), g1 + 2, c.sRed + (g1 & 1) * kRB + (c.L & 3) * 16 + 4 * c.q, z);
        rc.step_seq(bb, z, c.sRed + ((g1 + 1) & 1) * kRB, seq, g1 + 3, c.wv, c.q, c.L, c.sFlag + sl,
                    as_lane + sl * kD * kD, fa, ba);
      }
      SSTAMP(73, c.tid == 0);
    }
#endif
    __builtin_amdgcn_s_setprio(0);
    SSTAMP(80 + (c.wv & 15), c.lane == 0);
    if (fb + lay.fc < c.nf) __syncthreads();                    // B3: chunk done (not after the last)
  }
  // epilogue straight off the last frame: wait for every wave's last
  // partials (its sequence word), h = adj * h', store; no workgroup barrier
  // (the producers finish the metrics on their own, scene_producer)
  if (c.nf > 0) poll_seq_all(seq, c.nf + 2);
  SSTAMP(95, c.tid == 0);
  rc.store(a.h_out + (size_t)c.s * kD * H, H, c.wv, c.q, c.L, c.nf > 0 ? c.sRed + (c.nf & 1) * kRB : nullptr);
  SSTAMP(97, c.tid == 0);
}

// Role 2: the producers (waves 4..4+NP-1).
template <int NP, int MODE>
__device__ __forceinline__ void scene_producer(const StepArgs& a, const SceneLayout& lay,
                                               const SceneCtx& c) {
  constexpr int NT = 64 * (kRecW + NP);
  const int Nmax = a.d.Nmax, F = a.d.F, stride = a.d.stride;
  const int pw = c.wv - kRecW, L = c.L, q = c.q, lane = c.lane, s = c.s, ntiles = c.ntiles;
  const uint8_t* pm = a.ped_mask ? a.ped_mask + (size_t)s * Nmax : nullptr;
  // tile items of a chunk: item j -> frame j / ntiles, tile j % ntiles;
  // this producer takes items pw, pw + NP, ...  (k-th item: j = pw + k * NP)
  const int pp = lane >> 2, u = lane & 3;
  float2 tgA[3] = {}, tgB[3] = {};
  auto load_item = [&](int fb, int cnt, int k, float2 (&tg)[3]) {
    const int j = pw + k * NP;
    if (j >= cnt * ntiles) return;
    const int fl = j / ntiles, t = j - fl * ntiles;
    const int ne = 16 * t + pp;
    const int nc = ne < Nmax ? ne : 0;
    const float2* tp = reinterpret_cast<const float2*>(
        a.targets + (((size_t)s * F + fb + fl) * Nmax + nc) * kL2) + 3 * u;
    tg[0] = tp[0]; tg[1] = tp[1]; tg[2] = tp[2];
  };
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int fb = 0; fb < c.nf; fb += lay.fc) {
    const int cnt = (c.nf - fb) < lay.fc ? (c.nf - fb) : lay.fc;
    if (fb > 0) {
      if constexpr ((MODE & kModeDma16) != 0) scene_dma16<NT>(a, lay, c, fb, cnt, false);
      else scene_pos_dma<NT>(a, lay, c, fb, cnt);
    }
    scene_stage<NT, NP, 0>(a, lay, c, fb, cnt, [] {});
    load_item(fb, cnt, 0, tgA);       // first tiles' targets: in flight during the heads
    load_item(fb, cnt, 1, tgB);
    // Rm = Wr @ Rel, Rel = Ve * Ve (train.py:194-195, g2k_lstm_mcr.py:106):
    // rows t = 4q + i of column L, zero for t >= 8
    float rm[4];
    {
      const float ve0 = c.sV[lay.wcmax * kD + L], ve1 = c.sV[(lay.wcmax + 1) * kD + L];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int t = 4 * q + i;
        rm[i] = q < 2 ? fmaf(c.sm[SM_WR + 2 * t], ve0 * ve0, c.sm[SM_WR + 2 * t + 1] * (ve1 * ve1)) : 0.f;
      }
    }
    // phase 1 — the critical path: frame heads in frame order, M (and As
    // from chunk frame kRecW on: the recurrence waves head the first kRecW)
    // into the rings, then the frame's flags; the first heads the
    // recurrence will wait for get the issue priority
    for (int fl = pw; fl < cnt; fl += NP) {
      const int f = fb + fl;
      constexpr bool kHeads = (MODE & kOptRecHeads) != 0;
      const bool do_as = !kHeads || fl >= kRecW;
      if (kHeads ? (do_as && fl < 2 * kRecW) : fl < kRecW) __builtin_amdgcn_s_setprio(1);
      const FrameHeadOut hd =
          frame_head(c.sm, c.sV, c.sVG, fl * stride, lay.wcmax, rm, a.lambda, c.sRing + fl * kD * kD,
                     a.A_out ? a.A_out + ((size_t)s * F + f) * kD * kD : nullptr,
                     a.cost_out ? a.cost_out + ((size_t)s * F + f) * kT * kT : nullptr, L, q,
                     do_as);
      if (L < kL && q < 2) {
        float* m = c.sMring + fl * kL2 * kT;
        *reinterpret_cast<float4*>(m + L * kT + 4 * q) = make_float4(hd.mT0[0], hd.mT0[1], hd.mT0[2], hd.mT0[3]);
        *reinterpret_cast<float4*>(m + (kL + L) * kT + 4 * q) = make_float4(hd.mT1[0], hd.mT1[1], hd.mT1[2], hd.mT1[3]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) {
        lds_store_flag(c.sMflag + fl, f + 1);
        if (do_as) lds_store_flag(c.sFlag + fl, f + 1);
      }
      SSTAMP(3 + (f & 31), lane == 0);
      __builtin_amdgcn_s_setprio(0);
    }
    // phase 2 — predictions and errors, tiles spread over all producers
#ifdef G2K_DIAG_SKIP_TILES
    const int nitems = 0;   // diagnostic build only: no predictions / errors
#else
    const int nitems = cnt * ntiles > pw ? (cnt * ntiles - pw + NP - 1) / NP : 0;
#endif
    auto item = [&](int k, const float2 (&tg)[3]) {
      const int j = pw + k * NP;
      const int fl = j / ntiles, t = j - fl * ntiles;
      const int f = fb + fl;
      poll_flag(c.sMflag + fl, f + 1);         // M of this frame (maybe another producer's)
      float* pr = a.pred + ((size_t)s * F + f) * kL2 * Nmax;
      if constexpr ((MODE & kOptValuTiles) != 0)
        pred_tile(c.sMring + fl * kL2 * kT, c.sWo, pr, tg, pm, Nmax, c.nact, t, lane, acc);
      else
        pred_tile_mfma(c.sMring + fl * kL2 * kT, c.sWo, c.sY + pw * kD * kL2, pr, tg, pm, Nmax, c.nact,
                       t, L, q, lane, acc);
    };
    for (int k = 0; k < nitems; k += 2) {
      item(k, tgA);
      load_item(fb, cnt, k + 2, tgA);
      if (k + 1 < nitems) {
        item(k + 1, tgB);
        load_item(fb, cnt, k + 3, tgB);
      }
    }
    SSTAMP(80 + (c.wv & 15), lane == 0);
    if (fb + lay.fc < c.nf) __syncthreads();                    // B3: chunk done (not after the last)
  }
  if (pw == NP - 1) {
    // frames beyond n_frames: zero predictions (off the critical path)
    for (int i = lane; i < (F - c.nf) * kL2 * Nmax; i += 64)
      a.pred[((size_t)s * F + c.nf) * kL2 * Nmax + i] = 0.f;
  }
  // metrics: each producer publishes its partial sums, then takes a ticket
  // (LDS atomic); the wave drawing the last ticket sums the NP rows in
  // producer order (deterministic) and writes the scene's metrics row
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const float v = wave_sum(acc[k]);
    if (lane == 0) c.sMet[pw * 8 + k] = v;
  }
  int ticket = 0;
  if (lane == 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // partials before the ticket
    ticket = atomicAdd(c.sTicket, 1);
  }
  ticket = __builtin_amdgcn_readfirstlane(ticket);
  if (ticket == NP - 1 && lane < 8) {
    float v = 0.f;
    if (lane < 5) {
      if (c.nf > 0)
        for (int p = 0; p < NP; ++p) v += c.sMet[p * 8 + lane];
    } else if (lane == 5) {
      v = (float)c.nf;
    }
    a.metrics[(size_t)s * 8 + lane] = v;
  }
}

template <int TPW, int NP, int MODE>
__global__ void __launch_bounds__(64 * (kRecW + NP)) g2k_scene_kernel(StepArgs a, SceneLayout lay) {
  constexpr int NT = 64 * (kRecW + NP);
  constexpr int kRB = 16 * kRecW;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  SceneCtx c;
  c.s = blockIdx.x;
  c.tid = threadIdx.x; c.lane = c.tid & 63; c.wv = wave_id(); c.L = c.lane & 15; c.q = c.lane >> 4;
  const int Nmax = a.d.Nmax, F = a.d.F;
  c.ntiles = (Nmax + 15) >> 4;
  c.sWi = smem + lay.o_wi; c.sWo = smem + lay.o_wo; c.sVis = smem + lay.o_vis; c.sV = smem + lay.o_v;
  c.sm = smem + lay.o_small; c.sMet = smem + lay.o_met; c.sRing = smem + lay.o_ring;
  c.sMring = smem + lay.o_mring; c.sRed = smem + lay.o_red; c.sPos = smem + lay.o_pos;
  c.sVG = smem + lay.o_vg;
  c.sFlag = reinterpret_cast<int*>(smem + lay.o_flag);
  c.sMflag = reinterpret_cast<int*>(smem + lay.o_mflag);
  c.sY = smem + lay.o_y;
  c.sTicket = reinterpret_cast<int*>(c.sRed + 2 * kRB) + kRecW;
  SSTAMP_INIT();
#ifdef G2K_DIAG_TWICE
  // diagnostic build only: the whole scene twice in one launch (stamps of
  // the second pass overwrite the first: warm instruction cache / TLB)
  for (int pass = 0; pass < 2; ++pass) {
  __syncthreads();
#endif
  SSTAMP(0, c.tid == 0);
#ifdef G2K_STAMPS_SCENE
  if (c.lane == 0) {   // placement: HW_ID (SIMD_ID bits 5:4, CU_ID 11:8, SE_ID 15:13)
    unsigned hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    g2k_lds_stamps[60 + c.wv] = hw;
  }
  if (c.tid == 0) {
    unsigned long long rt;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt)::"memory");
    g2k_lds_stamps[98] = (unsigned)rt;
  }
#endif
  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;  // sequence words, ticket
  if (F > 0) {
    // issued before n_active / n_frames arrive: the first chunk's window for
    // min(F, fc) frames (a scene with fewer frames reads rows it ignores)
    const int wv = c.wv, lane = c.lane;
    SSTAMP(92, c.tid == 0 && F > 0);
    if constexpr ((MODE & kModeDma16) != 0) {
      scene_dma16<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc, true);
      SSTAMP(93, c.tid == 0);
    } else {
    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first
    SSTAMP(93, c.tid == 0);
    // the small segments: one wave each (one pointer per wave keeps the
    // kernel-argument loads off a serial s_load / s_waitcnt chain)
    for (int seg = wv; seg < 10; seg += NT / 64) {
      const float* src;
      float* dst;
      int n;
      switch (seg) {
        case 0: src = a.w.Wi; dst = c.sWi; n = Nmax * kD; break;
        case 1: src = a.w.Wo; dst = c.sWo; n = kT * Nmax; break;
        case 2: src = a.w.Wii; dst = c.sm + SM_WII; n = kD * kT; break;
        case 3: src = a.G + (size_t)c.s * kD * kT; dst = c.sm + SM_G; n = kD * kT; break;
        case 4: src = a.w.Wv; dst = c.sm + SM_WV; n = kT * (kD + 2); break;
        case 5: src = a.w.bv; dst = c.sm + SM_BV; n = kD; break;
        case 6: src = a.w.Wr; dst = c.sm + SM_WR; n = kT * 2; break;
        case 7: src = a.w.Wc; dst = c.sm + SM_WC; n = kL2 * kT; break;
        case 8: src = a.vislet + (size_t)c.s * 2 * Nmax; dst = c.sVis; n = Nmax; break;
        default: src = a.vislet + (size_t)c.s * 2 * Nmax + Nmax; dst = c.sVis + Nmax; n = Nmax; break;
      }
      for (int i = 0; i < n; i += 64)
        if (i + lane < n)
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i + lane),
                                           (__attribute__((address_space(3))) void*)(dst + i), 4, 0, 0);
    }
    }
    SSTAMP(94, c.tid == 0);
    if (c.tid < lay.fc) {                                // flags hold (global frame + 1)
      c.sFlag[c.tid] = 0;
      c.sMflag[c.tid] = 0;
    }
  }
  SSTAMP(103, c.tid == 0);
#ifdef G2K_DIAG_PROLOGUE
  // diagnostic build only: the prologue's loads, one barrier, nothing else
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (c.tid == 0) a.metrics[c.s * 8] = smem[c.lane];
  return;
#endif
  c.nact = clampi(a.n_active[c.s], 0, Nmax);
  c.nf = a.n_frames ? clampi(a.n_frames[c.s], 0, F) : F;
  SSTAMP(104, c.tid == 0 && c.nf >= 0);
  if (c.nf == 0) __syncthreads();   // no staging barrier will publish the initialised words
  if (c.wv < kRecW)
    scene_recurrence<TPW, NP, MODE>(a, lay, c);
  else
    scene_producer<NP, MODE>(a, lay, c);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup
  SSTAMP(100, c.tid == 0);
#ifdef G2K_STAMPS_SCENE
  if (c.tid == 0) {   // wall clock (100 MHz) beside the shader-clock stamps
    unsigned long long rt;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rt)::"memory");
    g2k_lds_stamps[99] = (unsigned)rt;
  }
#endif
#ifdef G2K_DIAG_TWICE
  }
#endif
  SSTAMP_FLUSH();
}

// ---------------------------------------------------------------------------
// g2k_lstm_mcr.forward() only (models/g2k_lstm_mcr.py:99-124), one WG / feed.
// ---------------------------------------------------------------------------
struct FwdArgs {
  g2k_dims d;
  g2k_weights w;
  const float* X;
  const float* Rel;
  const float* G;
  const int32_t* n_active;
  float* A_out;
  float* cost_out;
  float* pred;
  float lambda;
};

__global__ void __launch_bounds__(kNT) g2k_mcr_forward_kernel(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) float sX[(kD + 2) * kD];
  __shared__ float sE[kT * kD];
  __shared__ float sRm[kT * kD];
  __shared__ float sG[kD * kT];
  __shared__ float sC[kT * kT];
  __shared__ float sM[kL2 * kT];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int Nmax = a.d.Nmax;
  int nact = a.n_active[s];
  nact = nact < 0 ? 0 : (nact > Nmax ? Nmax : nact);
  for (int i = tid; i < (kD + 2) * kD; i += kNT) sX[i] = a.X[(size_t)s * (kD + 2) * kD + i];
  if (tid < kD * kT) sG[tid] = a.lambda * a.G[(size_t)s * kD * kT + tid];
  __syncthreads();
  if (tid < kT * kD) {
    const int t = tid >> 4, dcol = tid & 15;
    float e = 0.f;
    for (int k = 0; k < kD + 2; ++k) e = fmaf(a.w.Wv[t * (kD + 2) + k], sX[k * kD + dcol], e);
    sE[tid] = e + a.w.bv[dcol];
    const float* rel = a.Rel + (size_t)s * 2 * kD;
    sRm[tid] = fmaf(a.w.Wr[2 * t], rel[dcol], a.w.Wr[2 * t + 1] * rel[kD + dcol]);
  }
  __syncthreads();
  {
    const int r = tid >> 4, dcol = tid & 15;
    float x = 0.f;
    for (int t = 0; t < kT; ++t) x = fmaf(sG[r * kT + t], sE[t * kD + dcol] * sRm[t * kD + dcol], x);
    a.A_out[(size_t)s * kD * kD + tid] = x;
    if (tid < kT * kT) {
      const int t1 = tid >> 3, t2 = tid & 7;
      float c = 0.f;
      for (int k = 0; k < kD; ++k) c = fmaf(sE[t1 * kD + k], sG[k * kT + t2], c);
      sC[tid] = c;
      a.cost_out[(size_t)s * kT * kT + tid] = c;
    }
  }
  __syncthreads();
  if (tid < kL2 * kT) {
    const int jr = tid >> 3, t2 = tid & 7;
    float x = 0.f;
    for (int t = 0; t < kT; ++t) x = fmaf(a.w.Wc[jr * kT + t], sC[t * kT + t2], x);
    sM[tid] = x;
  }
  __syncthreads();
  for (int i = tid; i < kL2 * Nmax; i += kNT) {
    const int jr = i / Nmax, n = i - jr * Nmax;
    float x = 0.f;
    if (n < nact)
      for (int t = 0; t < kT; ++t) x = fmaf(sM[jr * kT + t], a.w.Wo[t * Nmax + n], x);
    a.pred[(size_t)s * kL2 * Nmax + i] = x;
  }
}

// ---------------------------------------------------------------------------
// Errors from predictions: variant 0 (train.py:640-674), 1 (sample.py:21-82)
// ---------------------------------------------------------------------------
struct ErrArgs {
  g2k_dims d;
  const float* pred;
  const float* targets;
  const int32_t* n_active;
  const int32_t* n_frames;
  const uint8_t* ped_mask;
  float* out;
};

__global__ void __launch_bounds__(kNT) g2k_errors_v0_kernel(ErrArgs a) {
  __shared__ float sMet[32];
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = wave_id();
  const int Nmax = a.d.Nmax, F = a.d.F;
  int nact = a.n_active[s];
  nact = nact < 0 ? 0 : (nact > Nmax ? Nmax : nact);
  int nf = a.n_frames ? a.n_frames[s] : F;
  nf = nf < 0 ? 0 : (nf > F ? F : nf);
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int task = tid; task < nf * Nmax; task += kNT) {
    const int f = task / Nmax, n = task - f * Nmax;
    if (n >= nact) continue;
    if (a.ped_mask && a.ped_mask[(size_t)s * Nmax + n] == 0) continue;
    float y[kL2];
    const float* pp = a.pred + ((size_t)s * F + f) * kL2 * Nmax + n;
#pragma unroll
    for (int jr = 0; jr < kL2; ++jr) y[jr] = pp[jr * Nmax];
    error_terms(y, a.targets + (((size_t)s * F + f) * Nmax + n) * kL2, acc);
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const float v = wave_sum(acc[k]);
    if (lane == 0) sMet[wv * 8 + k] = v;
  }
  __syncthreads();
  if (tid < 8) {
    float v = 0.f;
    if (tid < 5) v = (sMet[tid] + sMet[8 + tid]) + (sMet[16 + tid] + sMet[24 + tid]);
    else if (tid == 5) v = (float)nf;
    a.out[(size_t)s * 8 + tid] = v;
  }
}

// sample.py get_mean_error on one prediction per scene: i in [obs, L):
// e_i = sum_j (true - pred); ADE = mean_i(|e_i| / ((L-obs) N));
// FDE = mean_j(|true_{L-1,j} - pred_{L-1,j}| / N).
__global__ void __launch_bounds__(64) g2k_errors_v1_kernel(ErrArgs a) {
  const int s = blockIdx.x, lane = threadIdx.x;
  const int Nmax = a.d.Nmax, obs = a.d.T;
  int nact = a.n_active[s];
  nact = nact < 0 ? 0 : (nact > Nmax ? Nmax : nact);
  const float* pp = a.pred + (size_t)s * kL2 * Nmax;
  const float* tt = a.targets + (size_t)s * Nmax * kL2;
  float ex[kL], ey[kL];
#pragma unroll
  for (int l = 0; l < kL; ++l) { ex[l] = 0.f; ey[l] = 0.f; }
  float fsum = 0.f;
  for (int n = lane; n < nact; n += 64) {
#pragma unroll
    for (int l = 0; l < kL; ++l) {
      ex[l] += tt[n * kL2 + 2 * l] - pp[l * Nmax + n];
      ey[l] += tt[n * kL2 + 2 * l + 1] - pp[(kL + l) * Nmax + n];
    }
    const float dx = tt[n * kL2 + 2 * (kL - 1)] - pp[(kL - 1) * Nmax + n];
    const float dy = tt[n * kL2 + 2 * (kL - 1) + 1] - pp[(2 * kL - 1) * Nmax + n];
    fsum += sqrtf(fmaf(dx, dx, dy * dy));
  }
  float ade = 0.f;
  const float counter = (float)((kL - obs) * nact);
  for (int l = obs; l < kL; ++l) {
    const float x = wave_sum(ex[l]), y = wave_sum(ey[l]);
    ade += sqrtf(fmaf(x, x, y * y)) / counter;
  }
  fsum = wave_sum(fsum);
  if (lane < 8) {
    float v = 0.f;
    if (lane == 0) v = ade / (float)(kL - obs);
    else if (lane == 1) v = nact > 0 ? fsum / (float)nact / (float)nact : 0.f;
    else if (lane == 2) v = counter;
    a.out[(size_t)s * 8 + lane] = v;
  }
}

// ---------------------------------------------------------------------------
// nri_learned.py relation ops
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// nri_learned.py relation ops
// ---------------------------------------------------------------------------
__global__ void g2k_sigmoid_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = rcp(1.0f + __expf(-x[i]));
}

// one wave per row
__global__ void __launch_bounds__(64) g2k_row_softmax_kernel(const float* __restrict__ x,
                                                             float* __restrict__ y, int cols) {
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x;
  const float* xr = x + r * cols;
  float* yr = y + r * cols;
  float m = -INFINITY;
  for (int c = lane; c < cols; c += 64) m = fmaxf(m, xr[c]);
  for (int k = 32; k >= 1; k >>= 1) m = fmaxf(m, __shfl_xor(m, k, 64));
  float z = 0.f;
  for (int c = lane; c < cols; c += 64) z += __expf(xr[c] - m);
  z = wave_sum(z);
  const float rz = rcp(z);
  for (int c = lane; c < cols; c += 64) yr[c] = __expf(xr[c] - m) * rz;
}

// ---------------------------------------------------------------------------
// a6 GridLSTMCell (helper.py:31-39 vis/loc encoder, 131-141 static encoder):
// tf.contrib.rnn GridLSTMCell with share_time_frequency_weights,
// couple_input_forget_gates, frequency_skip == feature_size and a
// concatenated state; dataflow decoded from save/g2k_mcr_model_val_0.ckpt-0
// .meta (oracle/g2k_ref.py gridlstm_cell).  Rows are
// independent; a row's frequency blocks are a chain (block k reads block
// k - 1's c_freq, m_freq), so one lane owns one row and walks its blocks.
// W / b / peepholes are wave-uniform (scalar loads).  Elementwise and
// latency work on [rows, <= 32] tiles: no MFMA.
// ---------------------------------------------------------------------------
struct GridArgs {
  const float* in;
  const float* state;
  const float* W;      // [FS + 2U, 3U]
  const float* b;      // [3U]
  const float* peep;   // [4, U] = (wIf, wIt, wOf, wOt) or NULL
  float* out;          // [rows, K * 2U]
  float* state_out;    // [rows, K * 2U]
  int64_t rows, ld_in, ld_state;
  int K;
};

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + __expf(-x)); }

template <int U, int FS>
__global__ void __launch_bounds__(256) g2k_gridlstm_kernel(GridArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= a.rows) return;
  constexpr int NI = FS + 2 * U;
  const float* xr = a.in + r * a.ld_in;
  const float* sr = a.state + r * a.ld_state;
  float* orow = a.out + r * (int64_t)(2 * U) * a.K;
  float* srow = a.state_out + r * (int64_t)(2 * U) * a.K;
  const bool peep = a.peep != nullptr;
  float cf[U], mf[U];
#pragma unroll
  for (int j = 0; j < U; ++j) { cf[j] = 0.f; mf[j] = 0.f; }
  for (int k = 0; k < a.K; ++k) {
    float v[NI], ct[U];
#pragma unroll
    for (int i = 0; i < FS; ++i) v[i] = xr[k * FS + i];                 // x_k
#pragma unroll
    for (int j = 0; j < U; ++j) {
      ct[j] = sr[2 * U * k + j];                                         // c_time
      v[FS + j] = sr[2 * U * k + U + j];                                 // m_time
      v[FS + U + j] = mf[j];                                             // m_freq of block k - 1
    }
    float z[3 * U];
#pragma unroll
    for (int j = 0; j < 3 * U; ++j) {
      float acc = a.b[j];
#pragma unroll
      for (int i = 0; i < NI; ++i) acc = fmaf(v[i], a.W[i * 3 * U + j], acc);
      z[j] = acc;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      float gi = z[j];
      if (peep) gi += a.peep[j] * cf[j] + a.peep[U + j] * ct[j];
      const float ig = sigmoid_f(gi);                                    // coupled: f = 1 - i
      const float gg = tanhf(z[U + j]);
      const float cfn = (1.f - ig) * cf[j] + ig * gg;
      const float ctn = (1.f - ig) * ct[j] + ig * gg;
      float go = z[2 * U + j];
      if (peep) go += a.peep[2 * U + j] * cfn + a.peep[3 * U + j] * ctn;
      const float og = sigmoid_f(go);
      const float mfn = og * tanhf(cfn), mtn = og * tanhf(ctn);
      srow[2 * U * k + j] = ctn;
      srow[2 * U * k + U + j] = mtn;
      orow[2 * U * k + j] = mtn;
      orow[2 * U * k + U + j] = mfn;
      cf[j] = cfn;
      mf[j] = mfn;
    }
  }
}

// ---------------------------------------------------------------------------
// Train mode (SURVEY.md §8(d) "--mode train", §8(e) gradient all-reduce).
// The reference defines no loss or optimizer (SURVEY.md finding 5); the loss
// here is half the squared error of the pred_path_band rows against the
// targets the a9 errors use, over frames < n_frames and active, masked
// pedestrians, differentiated through a2-a4 and a7 (the a8 recurrence does
// not reach the predictions: Wr's gradient is exactly zero).  Restated in
// float64 by oracle/g2k_ref.py scene_loss_grad (pinned by finite
// differences).
//
// g2k_grad_kernel: grid (frame groups of GW, S), GW waves; wave w recomputes
// frame (group * GW + w)'s forward and back-propagates it through a dozen
// tiny products kept in its LDS scratch, one lane per output entry (every
// wave runs the same step sequence, so steps are separated by workgroup
// barriers).  The group's gradients are summed in wave order into the
// (scene, group) row of a partial buffer; two fixed-order reduction passes
// give the step's gradient.  Deterministic, no atomics.  VALU + LDS: each
// product is at most 24 x 16 outputs over an 8..Nmax contraction — too small
// for MFMA tiles to pay.
// ---------------------------------------------------------------------------
__host__ __device__ inline int grad_params(int Nmax) { return 24 * Nmax + 496; }

struct GradOff {
  int wi, wii, wv, bv, wr, wc, wo;
};
__host__ __device__ inline GradOff grad_off(int Nmax) {   // g2k_weights order
  GradOff o;
  o.wi = 0;
  o.wii = o.wi + Nmax * kD;
  o.wv = o.wii + kD * kT;
  o.bv = o.wv + kT * (kD + 2);
  o.wr = o.bv + kD;
  o.wc = o.wr + kT * 2;
  o.wo = o.wc + kL2 * kT;
  return o;
}

// rows that lanes walk in parallel (window norms, Wo, vislet) have the
// odd pitch Nmax + 1, so lanes on different rows hit different LDS banks
__host__ __device__ inline int grad_shared_floats(int Nmax) { return 26 * Nmax + 618; }
__host__ __device__ inline int grad_scratch_floats(int Nmax) { return 48 * Nmax + 2092; }
__host__ __device__ inline int grad_waves(int Nmax) { return Nmax > 128 ? 2 : 4; }
// launch width: grad_waves, or the G2K_GRAD_GW tuning override (1, 2, 4)
inline int grad_gw(int Nmax) {
  int GW = grad_waves(Nmax);
  if (const char* e = getenv("G2K_GRAD_GW")) {
    const int g = atoi(e);
    if (g == 1 || g == 2 || (g == 4 && Nmax <= 128)) GW = g;
  }
  return GW;
}
constexpr int kGradSlices = 32;

// one wave's LDS scratch in g2k_grad_kernel (floats)
struct GradScratch {
  float *pos, *tgt, *B, *X, *U, *E, *C, *M, *dM, *dC, *dE, *dX, *dU, *gWc, *gWv, *gbv, *gWii, *loss;
  __device__ GradScratch(float* p, int Nmax) {
    pos = p;  p += kT * 2 * Nmax;    // the frame's raw position window (LDS-DMA)
    tgt = p;  p += kL2 * Nmax;       // the frame's targets [Nmax][L][2] (LDS-DMA), then dY in place
    B = p;    p += kT * (Nmax + 1);  // window norms [T][Nmax + 1] (a2)
    X = p;    p += (kD + 2) * kD;    // [X0; Ve]
    U = p;    p += kT * kD;          // Bv @ Wi
    E = p;    p += kT * kD;
    C = p;    p += kT * kT;          // cost
    M = p;    p += kL2 * kT;         // Wc @ cost
    dM = p;   p += kL2 * kT;
    dC = p;   p += kT * kT;
    dE = p;   p += kT * kD;
    dX = p;   p += (kD + 2) * kD;
    dU = p;   p += kT * kD;
    gWc = p;  p += kL2 * kT;
    gWv = p;  p += kT * (kD + 2);
    gbv = p;  p += kD;
    gWii = p; p += kD * kT;
    loss = p;                        // {1/2 sum dY^2, count}
  }
};

struct GradArgs {
  g2k_dims d;
  g2k_weights w;
  const float *pos, *vislet, *G, *targets;
  const int32_t *n_active, *n_frames;
  const uint8_t* ped_mask;
  float lambda;
  float* part;   // [S * ngroup][P + 2]
  int ngroup;
};

// sum_{i < n} x[i] * y[i * ys] with four independent accumulators (the LDS
// loads of four terms are in flight together)
__device__ __forceinline__ float dot_strided(const float* x, const float* y, int ys, int n) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    a0 = fmaf(x[i], y[i * ys], a0);
    a1 = fmaf(x[i + 1], y[(i + 1) * ys], a1);
    a2 = fmaf(x[i + 2], y[(i + 2) * ys], a2);
    a3 = fmaf(x[i + 3], y[(i + 3) * ys], a3);
  }
  for (; i < n; ++i) a0 = fmaf(x[i], y[i * ys], a0);
  return (a0 + a1) + (a2 + a3);
}

// LDS hand-off between the lanes of ONE wave: DS instructions of a wave
// complete in issue order, so only compiler reordering has to be fenced
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int GW>
__global__ void __launch_bounds__(64 * GW) g2k_grad_kernel(GradArgs a) {
  constexpr int NT = 64 * GW;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Nmax = a.d.Nmax, F = a.d.F, P = grad_params(Nmax);
  const int s = blockIdx.y, grp = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
  const int f = grp * GW + wv;
  STAMP(18);
  float* sWi = smem;
  float* sWo = sWi + Nmax * kD;
  const int NP1 = Nmax + 1;
  float* sWii = sWo + kT * NP1;
  float* sWv = sWii + kD * kT;
  float* sbv = sWv + kT * (kD + 2);
  float* sWc = sbv + kD;
  float* sg = sWc + kL2 * kT;
  float* sVis = sg + kD * kT;
  float* scratch0 = smem + grad_shared_floats(Nmax);
  const int PW = grad_scratch_floats(Nmax);
  const GradScratch w(scratch0 + wv * PW, Nmax);
  const uint8_t* pm = a.ped_mask ? a.ped_mask + (size_t)s * Nmax : nullptr;

  // every global byte by 4-byte LDS-DMA, all in flight before n_active /
  // n_frames are known and before any use (one vmcnt wait): weights, G and
  // vislet per workgroup; each wave its frame's position window and targets
  dma4_copy_t<NT>(a.w.Wi, sWi, Nmax * kD, wv, lane);
  for (int t = 0; t < kT; ++t) dma4_copy_t<NT>(a.w.Wo + t * Nmax, sWo + t * NP1, Nmax, wv, lane);
  dma4_copy_t<NT>(a.w.Wii, sWii, kD * kT, wv, lane);
  dma4_copy_t<NT>(a.w.Wv, sWv, kT * (kD + 2), wv, lane);
  dma4_copy_t<NT>(a.w.bv, sbv, kD, wv, lane);
  dma4_copy_t<NT>(a.w.Wc, sWc, kL2 * kT, wv, lane);
  dma4_copy_t<NT>(a.G + (size_t)s * kD * kT, sg, kD * kT, wv, lane);   // lambda applied at use
  for (int j = 0; j < 2; ++j)
    dma4_copy_t<NT>(a.vislet + ((size_t)s * 2 + j) * Nmax, sVis + j * NP1, Nmax, wv, lane);
  if (f < F) {
    for (int t = 0; t < kT; ++t)
      dma4_copy_t<64>(a.pos + ((size_t)s * a.d.W + (size_t)f * a.d.stride + t) * Nmax * 2,
                      w.pos + t * 2 * Nmax, 2 * Nmax, 0, lane);
    dma4_copy_t<64>(a.targets + ((size_t)s * F + f) * Nmax * kL2, w.tgt, kL2 * Nmax, 0, lane);
  }
  const int nact = clampi(a.n_active[s], 0, Nmax);
  const int nf = a.n_frames ? clampi(a.n_frames[s], 0, F) : F;
  const bool act = f < nf;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  STAMP(19);
  for (int i = lane; i < kT * Nmax; i += 64) {                 // a2 window norms (train.py:76-85)
    const int t = i / Nmax, n = i - t * Nmax;
    const float2 p = *reinterpret_cast<const float2*>(w.pos + t * 2 * Nmax + 2 * n);
    w.B[t * NP1 + n] = (act && n < nact) ? sqrtf(fmaf(p.x, p.x, p.y * p.y)) : 0.f;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(20);
  // forward (train.py:178-195, models/g2k_lstm_mcr.py:105-122)
  for (int o = lane; o < (kT + 2) * kD; o += 64) {           // U = Bv @ Wi; Ve = vislet @ Wi
    const int r = o >> 4, d = o & 15;
    const float* src = r < kT ? w.B + r * NP1 : sVis + (r - kT) * NP1;
    const float acc = dot_strided(src, sWi + d, kD, nact);
    if (r < kT) w.U[r * kD + d] = acc;
    else w.X[(kD + r - kT) * kD + d] = acc;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(21);
  for (int o = lane; o < kD * kD; o += 64) {                  // X0 = Wii @ U
    const int r = o >> 4, d = o & 15;
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < kT; ++t) acc = fmaf(sWii[r * kT + t], w.U[t * kD + d], acc);
    w.X[o] = acc;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(22);
  for (int o = lane; o < kT * kD; o += 64) {                  // E = Wv @ X + bv
    const int t = o >> 4, d = o & 15;
    float acc = sbv[d];
#pragma unroll
    for (int c = 0; c < kD + 2; ++c) acc = fmaf(sWv[t * (kD + 2) + c], w.X[c * kD + d], acc);
    w.E[o] = acc;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(23);
  {                                                           // cost = E @ (lambda G)
    const int t = lane >> 3, u = lane & 7;
    float acc = 0.f;
#pragma unroll
    for (int d = 0; d < kD; ++d) acc = fmaf(w.E[t * kD + d], sg[d * kT + u], acc);
    w.C[lane] = a.lambda * acc;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(24);
  for (int o = lane; o < kL2 * kT; o += 64) {                 // M = Wc @ cost
    const int r = o >> 3, t = o & 7;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < kT; ++u) acc = fmaf(sWc[r * kT + u], w.C[u * kT + t], acc);
    w.M[o] = acc;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(25);
  // dY = Y - target on active, masked pedestrians (Y = M @ Wo, :122-124)
  float lsum = 0.f;
  for (int o = lane; o < kL2 * Nmax; o += 64) {     // o walks targets[n][l][x|y]
    const int n = o / kL2, rem = o - n * kL2, l = rem >> 1;
    const int r = (rem & 1) ? kL + l : l;
    float dy = 0.f;
    if (act && n < nact && (pm ? pm[n] != 0 : true)) {
      const float tg = w.tgt[o];
      float y = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) y = fmaf(w.M[r * kT + t], sWo[t * NP1 + n], y);
      dy = y - tg;
      lsum = fmaf(dy, dy, lsum);
    }
    w.tgt[o] = dy;                                    // dY(r, n), in place
  }
  float cnt = 0.f;
  for (int n = lane; n < Nmax; n += 64) cnt += (act && n < nact && (pm ? pm[n] != 0 : true)) ? 1.f : 0.f;
  lsum = wave_sum(lsum);
  cnt = wave_sum(cnt);
  if (lane == 0) {
    w.loss[0] = 0.5f * lsum;
    w.loss[1] = cnt;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(26);
  // backward
  for (int o = lane; o < kL2 * kT; o += 64) {                 // dM = dY @ Wo^T
    const int r = o >> 3, t = o & 7;
    const float* dy = w.tgt + ((r < kL) ? 2 * r : 2 * (r - kL) + 1);   // dY(r, n) at dy[24 n]
    const float* wo = sWo + t * NP1;
    float a0 = 0.f, a1 = 0.f;
    int n = 0;
    for (; n + 2 <= nact; n += 2) {
      a0 = fmaf(dy[n * kL2], wo[n], a0);
      a1 = fmaf(dy[(n + 1) * kL2], wo[n + 1], a1);
    }
    if (n < nact) a0 = fmaf(dy[n * kL2], wo[n], a0);
    w.dM[o] = a0 + a1;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(27);
  for (int o = lane; o < kT * kT + kL2 * kT; o += 64) {
    if (o < kT * kT) {                                        // dcost = Wc^T @ dM
      const int u = o >> 3, t = o & 7;
      float acc = 0.f;
      for (int r = 0; r < kL2; ++r) acc = fmaf(sWc[r * kT + u], w.dM[r * kT + t], acc);
      w.dC[o] = acc;
    } else {                                                  // dWc = dM @ cost^T
      const int p = o - kT * kT, r = p >> 3, u = p & 7;
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) acc = fmaf(w.dM[r * kT + t], w.C[u * kT + t], acc);
      w.gWc[p] = acc;
    }
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(28);
  for (int o = lane; o < kT * kD; o += 64) {                  // dE = dcost @ (lambda G)^T
    const int t = o >> 4, d = o & 15;
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < kT; ++u) acc = fmaf(w.dC[t * kT + u], sg[d * kT + u], acc);
    w.dE[o] = a.lambda * acc;
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(29);
  for (int o = lane; o < (kD + 2) * kD + kT * (kD + 2) + kD; o += 64) {
    if (o < (kD + 2) * kD) {                                  // dX = Wv^T @ dE
      const int c = o >> 4, d = o & 15;
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) acc = fmaf(sWv[t * (kD + 2) + c], w.dE[t * kD + d], acc);
      w.dX[o] = acc;
    } else if (o < (kD + 2) * kD + kT * (kD + 2)) {           // dWv = dE @ X^T
      const int p = o - (kD + 2) * kD, t = p / (kD + 2), c = p - t * (kD + 2);
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < kD; ++d) acc = fmaf(w.dE[t * kD + d], w.X[c * kD + d], acc);
      w.gWv[p] = acc;
    } else {                                                  // dbv = column sums of dE
      const int d = o - (kD + 2) * kD - kT * (kD + 2);
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) acc += w.dE[t * kD + d];
      w.gbv[d] = acc;
    }
  }
  wave_lds_sync();   // the wave's own scratch only
  STAMP(30);
  for (int o = lane; o < 2 * kT * kD; o += 64) {
    if (o < kT * kD) {                                        // dU = Wii^T @ dX0
      const int t = o >> 4, d = o & 15;
      float acc = 0.f;
#pragma unroll
      for (int r = 0; r < kD; ++r) acc = fmaf(sWii[r * kT + t], w.dX[r * kD + d], acc);
      w.dU[o] = acc;
    } else {                                                  // dWii = dX0 @ U^T
      const int p = o - kT * kD, r = p >> 3, t = p & 7;
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < kD; ++d) acc = fmaf(w.dX[r * kD + d], w.U[t * kD + d], acc);
      w.gWii[p] = acc;
    }
  }
  __syncthreads();
  STAMP(31);
  // this group's gradient row, frames summed in wave order
  const GradOff go = grad_off(Nmax);
  float* row = a.part + ((size_t)s * a.ngroup + grp) * (size_t)(P + 2);
  for (int p = tid; p < P + 2; p += NT) {
    float v = 0.f;
    for (int wi = 0; wi < GW; ++wi) {
      const GradScratch x(scratch0 + wi * PW, Nmax);
      float c = 0.f;
      if (p < go.wii) {                                       // dWi = Bv^T @ dU + vislet^T @ dVe
        const int n = p >> 4, d = p & 15;
        if (n < nact) {
#pragma unroll
          for (int t = 0; t < kT; ++t) c = fmaf(x.B[t * NP1 + n], x.dU[t * kD + d], c);
          c = fmaf(sVis[n], x.dX[kD * kD + d], c);
          c = fmaf(sVis[NP1 + n], x.dX[(kD + 1) * kD + d], c);
        }
      } else if (p < go.wv) {
        c = x.gWii[p - go.wii];
      } else if (p < go.bv) {
        c = x.gWv[p - go.wv];
      } else if (p < go.wr) {
        c = x.gbv[p - go.bv];
      } else if (p < go.wc) {
        c = 0.f;                                              // Wr does not reach pred
      } else if (p < go.wo) {
        c = x.gWc[p - go.wc];
      } else if (p < P) {                                     // dWo = M^T @ dY
        const int q = p - go.wo, t = q / Nmax, n = q - t * Nmax;
        for (int r = 0; r < kL2; ++r)
          c = fmaf(x.M[r * kT + t], x.tgt[n * kL2 + ((r < kL) ? 2 * r : 2 * (r - kL) + 1)], c);
      } else {
        c = x.loss[p - P];
      }
      v += c;
    }
    row[p] = v;
  }
  STAMP(32);
}

// g2k_grad_seq_kernel: the same per-frame products, but ONE frame at a time
// over all 256 threads of the workgroup (four times shorter phases), the
// group's frames in sequence with the next frame's position window and
// targets prefetched by LDS-DMA under the current frame's work, and the
// group's row accumulated in LDS by the thread that owns each entry (frame
// order: the same sums as g2k_grad_kernel's wave-order sum).  One scratch
// instead of one per wave: ~34 KB of LDS at Nmax = 32, four workgroups per
// CU, so every (scene, group) of eth_hotel_synth (5 frames each) is resident
// at once.
// workgroups per CU the register budget allows (one wave per SIMD each)
constexpr int kGradSeqWgPerCu = 5;
__host__ __device__ inline int grad_seq_buf_floats(int Nmax) { return (2 * kT + kL2) * Nmax; }
__host__ __device__ inline int grad_seq_lds_floats(int Nmax) {
  return grad_shared_floats(Nmax) + grad_scratch_floats(Nmax) + 8 + grad_seq_buf_floats(Nmax)
         + grad_params(Nmax) + 2 + Nmax + 4 * 256;
}
// frames per workgroup: the workgroups run in ceil(groups / slots) rounds of
// `fpg` sequential frames each (slots = CUs x resident workgroups per CU, by
// LDS and by the register bound kGradSeqWgPerCu); minimise rounds x fpg,
// ties to the larger fpg (fewer prologues and partial rows)
static int grad_cu_count() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1)
      n = 256;
    cus = n;
  }
  return cus;
}
inline int grad_seq_fpg(const g2k_dims* d) {
  if (const char* e = getenv("G2K_GRAD_FPG")) {              // tuning override
    const int v = atoi(e);
    if (v >= 1 && v <= 64) return v;
  }
  int per_cu = (160 * 1024) / (4 * grad_seq_lds_floats(d->Nmax));
  per_cu = per_cu < 1 ? 1 : (per_cu > kGradSeqWgPerCu ? kGradSeqWgPerCu : per_cu);
  const int64_t slots = (int64_t)grad_cu_count() * per_cu;
  int best = 1;
  int64_t best_cost = -1;
  for (int fpg = 1; fpg <= (d->F < 32 ? d->F : 32); ++fpg) {
    const int64_t groups = (int64_t)d->S * ((d->F + fpg - 1) / fpg);
    const int64_t cost = ((groups + slots - 1) / slots) * fpg;
    if (best_cost < 0 || cost <= best_cost) { best = fpg; best_cost = cost; }
  }
  return best;
}

// WPE: resident workgroups per CU the build targets (one wave per SIMD each):
// kGradSeqWgPerCu when LDS allows that many, else 2 (LDS admits fewer
// workgroups anyway), which leaves registers for independent MFMA chains in
// the K = n products
template <int WPE>
__global__ void __launch_bounds__(256, WPE) g2k_grad_seq_kernel(GradArgs a, int fpg) {
  constexpr int kChains = WPE >= kGradSeqWgPerCu ? 1 : 4;
  constexpr int NT = 256;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int Nmax = a.d.Nmax, F = a.d.F, P = grad_params(Nmax), P2 = P + 2;
  const int s = blockIdx.y, grp = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = wave_id();
  const int NP1 = Nmax + 1;
  float* sWi = smem;
  float* sWo = sWi + Nmax * kD;
  float* sWii = sWo + kT * NP1;
  float* sWv = sWii + kD * kT;
  float* sbv = sWv + kT * (kD + 2);
  float* sWc = sbv + kD;
  float* sg = sWc + kL2 * kT;
  float* sVis = sg + kD * kT;
  float* scr = smem + grad_shared_floats(Nmax);
  GradScratch w(scr, Nmax);
  float* sLoss = scr + grad_scratch_floats(Nmax);     // [4 waves][loss, count]
  float* buf[2] = {w.pos, sLoss + 8};                 // pos window then targets, per frame
  float* racc = buf[1] + grad_seq_buf_floats(Nmax);  // [P + 2] this group's row
  float* sAct = racc + P2;                            // [Nmax] 1 for active, masked pedestrians
  float* sUp = sAct + Nmax;                           // [4 waves][16][16] partial U/Ve tiles
  const int f0 = grp * fpg;
  const int L16 = lane & 15, q4 = lane >> 4;          // MFMA 16x16x4 lane roles
  const int ntile = (Nmax + 15) >> 4;                 // 16-pedestrian tiles
  STAMP(18);

  dma4_copy_t<NT>(a.w.Wi, sWi, Nmax * kD, wv, lane);
  for (int t = 0; t < kT; ++t) dma4_copy_t<NT>(a.w.Wo + t * Nmax, sWo + t * NP1, Nmax, wv, lane);
  dma4_copy_t<NT>(a.w.Wii, sWii, kD * kT, wv, lane);
  dma4_copy_t<NT>(a.w.Wv, sWv, kT * (kD + 2), wv, lane);
  dma4_copy_t<NT>(a.w.bv, sbv, kD, wv, lane);
  dma4_copy_t<NT>(a.w.Wc, sWc, kL2 * kT, wv, lane);
  dma4_copy_t<NT>(a.G + (size_t)s * kD * kT, sg, kD * kT, wv, lane);   // lambda applied at use
  for (int j = 0; j < 2; ++j)
    dma4_copy_t<NT>(a.vislet + ((size_t)s * 2 + j) * Nmax, sVis + j * NP1, Nmax, wv, lane);
  auto dma_frame = [&](int f, float* dst) {
    for (int t = 0; t < kT; ++t)
      dma4_copy_t<NT>(a.pos + ((size_t)s * a.d.W + (size_t)f * a.d.stride + t) * Nmax * 2,
                      dst + t * 2 * Nmax, 2 * Nmax, wv, lane);
    dma4_copy_t<NT>(a.targets + ((size_t)s * F + f) * Nmax * kL2, dst + kT * 2 * Nmax, kL2 * Nmax,
                    wv, lane);
  };
  if (f0 < F) dma_frame(f0, buf[0]);
  const int nact = clampi(a.n_active[s], 0, Nmax);
  const int nf = a.n_frames ? clampi(a.n_frames[s], 0, F) : F;
  // frames past n_frames contribute exactly zero (their dY is masked)
  const int nfg = max(0, min(fpg, min(nf, F) - f0));
  const uint8_t* pm = a.ped_mask ? a.ped_mask + (size_t)s * Nmax : nullptr;
  for (int n = tid; n < Nmax; n += NT) sAct[n] = (n < nact && (pm ? pm[n] != 0 : true)) ? 1.f : 0.f;
  for (int p = tid; p < P2; p += NT) racc[p] = 0.f;
  const GradOff go = grad_off(Nmax);
  // the weights enter each frame only through K1 = Wv[:, :16] @ Wii (E = K1 U
  // + Wv[:, 16:] Ve + bv, dU = K1^T dE), so the weight-side gradients need
  // only sums over the group's frames, expanded once after the loop:
  //   dWv[:, :16] = (sum dE U^T) Wii^T   dWii = Wv[:, :16]^T (sum dE U^T)
  //   dWv[:, 16:] = (sum dE) Ve^T        dbv = column sums of (sum dE)
  //   dWi += vislet^T (Wv[:, 16:]^T sum dE)
  // They live in the X0 block of the scratch (X0 itself is never formed).
  float* sK1 = w.X;                                   // [T][T]
  float* sAU = w.X + kT * kT;                         // [T][T]  sum dE U^T
  float* sSE = w.X + 2 * kT * kT;                     // [T][D]  sum dE
  for (int o = tid; o < kT * kT + kT * kD; o += NT) sAU[o] = 0.f;

  for (int k = 0; k < nfg; ++k) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                  // frame k landed; frame k - 1 done
    STAMP(19);
    w.pos = buf[k & 1];
    w.tgt = w.pos + kT * 2 * Nmax;
    if (k + 1 < nfg) dma_frame(f0 + k + 1, buf[(k + 1) & 1]);
    if (Nmax >= NT / 2) {                             // a2 window norms (train.py:76-85):
      for (int n = tid; n < Nmax; n += NT) {          // one pedestrian per thread when wide,
#pragma unroll 4
        for (int t = 0; t < kT; ++t) {
          const float2 q = *reinterpret_cast<const float2*>(w.pos + t * 2 * Nmax + 2 * n);
          w.B[t * NP1 + n] = n < nact ? sqrtf(fmaf(q.x, q.x, q.y * q.y)) : 0.f;
        }
      }
    } else {
      for (int i = tid; i < kT * Nmax; i += NT) {     // else (frame row, pedestrian) pairs
        const int t = i / Nmax, n = i - t * Nmax;
        const float2 q = *reinterpret_cast<const float2*>(w.pos + t * 2 * Nmax + 2 * n);
        w.B[t * NP1 + n] = n < nact ? sqrtf(fmaf(q.x, q.x, q.y * q.y)) : 0.f;
      }
    }
    if (k == 0 && tid < kT * kT) {                    // K1 = Wv[:, :16] @ Wii
      const int t = tid >> 3, u = tid & 7;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < kD; ++c) acc = fmaf(sWv[t * (kD + 2) + c], sWii[c * kT + u], acc);
      sK1[tid] = acc;
    }
    __syncthreads();
    STAMP(20);
    {                                                 // U = Bv @ Wi; Ve = vislet @ Wi (MFMA:
      f32x4 accs[kChains];                           // rows r < 10 of one 16 x 16 tile, the
      const float* arow = L16 < kT ? w.B + L16 * NP1 // K = n steps split over the waves)
                                   : sVis + (L16 < kT + 2 ? L16 - kT : 0) * NP1;
#pragma unroll
      for (int j = 0; j < kChains; ++j) accs[j] = {0.f, 0.f, 0.f, 0.f};
      for (int n0 = 4 * wv; n0 < nact; n0 += 64) {    // four k-steps' loads in flight
        float av[4], bv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + 16 * j + q4;
          const bool ok = n < nact;
          av[j] = (ok && L16 < kT + 2) ? arow[n] : 0.f;
          bv[j] = ok ? sWi[n * kD + L16] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) accs[j % kChains] = mfma4(av[j], bv[j], accs[j % kChains]);
      }
      f32x4 acc = accs[0];
#pragma unroll
      for (int j = 1; j < kChains; ++j) acc += accs[j];
#pragma unroll
      for (int v = 0; v < 4; ++v) sUp[wv * 256 + (4 * q4 + v) * 16 + L16] = acc[v];
    }
    __syncthreads();
    STAMP(21);
    // the waves' partial tiles summed in wave order (one rounding for everyone)
    auto usum = [&](int o) { return ((sUp[o] + sUp[256 + o]) + sUp[512 + o]) + sUp[768 + o]; };
    if (tid < kT * kD) {                              // E = K1 @ U + Wv[:, 16:] @ Ve + bv
      const int t = tid >> 4, d = tid & 15;
      float acc = sbv[d];
#pragma unroll
      for (int u = 0; u < kT; ++u) acc = fmaf(sK1[t * kT + u], usum(u * kD + d), acc);
      acc = fmaf(sWv[t * (kD + 2) + kD], usum(kD * kT + d), acc);
      acc = fmaf(sWv[t * (kD + 2) + kD + 1], usum(kD * (kT + 1) + d), acc);
      w.E[tid] = acc;
    } else {                                          // U, and Ve into X rows 16, 17
      const int o = tid - kT * kD;
      w.U[o] = usum(o);
      if (o < 2 * kD) w.X[kD * kD + o] = usum(kD * kT + o);
    }
    __syncthreads();
    STAMP(22);
    if (tid < kT * kT) {                              // cost = E @ (lambda G)
      const int t = tid >> 3, u = tid & 7;
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < kD; ++d) acc = fmaf(w.E[t * kD + d], sg[d * kT + u], acc);
      w.C[tid] = a.lambda * acc;
    }
    __syncthreads();
    STAMP(24);
    if (tid < kL2 * kT) {                             // M = Wc @ cost
      const int r = tid >> 3, t = tid & 7;
      float acc = 0.f;
#pragma unroll
      for (int u = 0; u < kT; ++u) acc = fmaf(sWc[r * kT + u], w.C[u * kT + t], acc);
      w.M[tid] = acc;
    }
    __syncthreads();
    STAMP(25);
    // dY = Y - target on active, masked pedestrians (Y = M @ Wo, :122-124)
    float lsum = 0.f, cnt = 0.f;
    for (int it = wv; it < 2 * ntile; it += 4) {      // Y tiles (MFMA): rows r, 16 pedestrians
      const int rt = it & 1, n = (it >> 1) * 16 + L16;
      const int ra = rt * 16 + L16;                   // A row of this lane
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int t = 4 * ks + q4;
        const float av = ra < kL2 ? w.M[ra * kT + t] : 0.f;
        const float bv = n < Nmax ? sWo[t * NP1 + n] : 0.f;
        acc = mfma4(av, bv, acc);
      }
      if (n < Nmax) {
        const bool on = sAct[n] != 0.f;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int r = rt * 16 + 4 * q4 + v;
          if (r < kL2) {
            const int o = n * kL2 + ((r < kL) ? 2 * r : 2 * (r - kL) + 1);
            float dy = 0.f;
            if (on) {
              dy = acc[v] - w.tgt[o];
              lsum = fmaf(dy, dy, lsum);
            }
            w.tgt[o] = dy;                            // dY(r, n), in place
          }
        }
      }
    }
    for (int n = tid; n < Nmax; n += NT) cnt += sAct[n];
    lsum = wave_sum(lsum);
    cnt = wave_sum(cnt);
    if (lane == 0) {
      sLoss[2 * wv] = 0.5f * lsum;
      sLoss[2 * wv + 1] = cnt;
    }
    __syncthreads();
    STAMP(26);
    if (wv < 2) {                                     // dM = dY @ Wo^T (MFMA, K = n)
      const int ra = wv * 16 + L16;
      const int oa = ra < kL2 ? ((ra < kL) ? 2 * ra : 2 * (ra - kL) + 1) : 0;
      f32x4 accs[kChains];                            // independent MFMA chains (wide builds)
#pragma unroll
      for (int j = 0; j < kChains; ++j) accs[j] = {0.f, 0.f, 0.f, 0.f};
      for (int n0 = 0; n0 < nact; n0 += 16) {         // four k-steps' loads in flight
        float av[4], bv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + 4 * j + q4;
          const bool ok = n < nact;
          av[j] = (ok && ra < kL2) ? w.tgt[n * kL2 + oa] : 0.f;
          bv[j] = (ok && L16 < kT) ? sWo[L16 * NP1 + n] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) accs[j % kChains] = mfma4(av[j], bv[j], accs[j % kChains]);
      }
      f32x4 acc = accs[0];
#pragma unroll
      for (int j = 1; j < kChains; ++j) acc += accs[j];
      if (L16 < kT) {
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int r = wv * 16 + 4 * q4 + v;
          if (r < kL2) w.dM[r * kT + L16] = acc[v];
        }
      }
    } else {                                          // dWo += M^T @ dY (MFMA, K = r)
      for (int nt = wv - 2; nt < ntile; nt += 2) {
        const int n = nt * 16 + L16;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < kL2 / 4; ++ks) {
          const int r = 4 * ks + q4;
          const float av = L16 < kT ? w.M[r * kT + L16] : 0.f;
          const float bv = n < Nmax ? w.tgt[n * kL2 + ((r < kL) ? 2 * r : 2 * (r - kL) + 1)] : 0.f;
          acc = mfma4(av, bv, acc);
        }
        if (q4 < 2 && n < Nmax) {
#pragma unroll
          for (int v = 0; v < 4; ++v) racc[go.wo + (4 * q4 + v) * Nmax + n] += acc[v];
        }
      }
    }
    __syncthreads();
    STAMP(27);
    if (tid < kT * kT) {                              // dcost = Wc^T @ dM
      const int u = tid >> 3, t = tid & 7;
      float acc = 0.f;
      for (int r = 0; r < kL2; ++r) acc = fmaf(sWc[r * kT + u], w.dM[r * kT + t], acc);
      w.dC[tid] = acc;
    } else {                                          // dWc = dM @ cost^T (192 outputs)
      const int p = tid - kT * kT, r = p >> 3, u = p & 7;
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) acc = fmaf(w.dM[r * kT + t], w.C[u * kT + t], acc);
      w.gWc[p] = acc;
    }
    __syncthreads();
    STAMP(28);
    if (tid < kT * kD) {                              // dE = dcost @ (lambda G)^T
      const int t = tid >> 4, d = tid & 15;
      float acc = 0.f;
#pragma unroll
      for (int u = 0; u < kT; ++u) acc = fmaf(w.dC[t * kT + u], sg[d * kT + u], acc);
      w.dE[tid] = a.lambda * acc;
    }
    __syncthreads();
    STAMP(29);
    if (tid < kT * kD) {                              // dU = K1^T @ dE
      const int u = tid >> 4, d = tid & 15;
      float acc = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) acc = fmaf(sK1[t * kT + u], w.dE[t * kD + d], acc);
      w.dU[tid] = acc;
    } else {
      const int o = tid - kT * kD;                    // 0..127
      sSE[o] += w.dE[o];                              // sum dE
      if (o < kT * kT) {                              // sum dE U^T
        const int t = o >> 3, u = o & 7;
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < kD; ++d) acc = fmaf(w.dE[t * kD + d], w.U[u * kD + d], acc);
        sAU[o] += acc;
      }
    }
    __syncthreads();
    STAMP(30);
    for (int nt = wv; nt < ntile; nt += 4) {          // dWi += Bv^T @ dU (MFMA)
      const int na = nt * 16 + L16;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {                // the 8 window rows
        const int kk = 4 * ks + q4;
        const float av = na < nact ? w.B[kk * NP1 + na] : 0.f;
        acc = mfma4(av, w.dU[kk * kD + L16], acc);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int n = nt * 16 + 4 * q4 + v;
        if (n < Nmax) racc[go.wi + n * kD + L16] += acc[v];
      }
    }
    for (int p = tid; p < kL2 * kT + 2; p += NT) {    // dWc, loss and count of this frame
      if (p < kL2 * kT) {
        racc[go.wc + p] += w.gWc[p];
      } else {
        const int j = p - kL2 * kT;                   // waves in order
        racc[P + j] += ((sLoss[j] + sLoss[2 + j]) + sLoss[4 + j]) + sLoss[6 + j];
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA outlives the workgroup
  __syncthreads();
  if (nfg > 0) {                                      // the weight-side gradients of the group
    float* sdVe = w.dX;                               // [2][D] Wv[:, 16:]^T sum dE
    for (int o = tid; o < kT * (kD + 2) + kD * kT + kD + 2 * kD; o += NT) {
      float acc = 0.f;
      if (o < kT * (kD + 2)) {                        // dWv
        const int t = o / (kD + 2), c = o - t * (kD + 2);
        if (c < kD) {
#pragma unroll
          for (int u = 0; u < kT; ++u) acc = fmaf(sAU[t * kT + u], sWii[c * kT + u], acc);
        } else {
#pragma unroll
          for (int d = 0; d < kD; ++d) acc = fmaf(sSE[t * kD + d], w.X[c * kD + d], acc);
        }
        racc[go.wv + o] = acc;
      } else if (o < kT * (kD + 2) + kD * kT) {       // dWii
        const int q = o - kT * (kD + 2), c = q >> 3, u = q & 7;
#pragma unroll
        for (int t = 0; t < kT; ++t) acc = fmaf(sWv[t * (kD + 2) + c], sAU[t * kT + u], acc);
        racc[go.wii + q] = acc;
      } else if (o < kT * (kD + 2) + kD * kT + kD) {  // dbv
        const int d = o - kT * (kD + 2) - kD * kT;
#pragma unroll
        for (int t = 0; t < kT; ++t) acc += sSE[t * kD + d];
        racc[go.bv + d] = acc;
      } else {                                        // dVe
        const int q = o - kT * (kD + 2) - kD * kT - kD, j = q >> 4, d = q & 15;
#pragma unroll
        for (int t = 0; t < kT; ++t) acc = fmaf(sWv[t * (kD + 2) + kD + j], sSE[t * kD + d], acc);
        sdVe[q] = acc;
      }
    }
    __syncthreads();
    for (int p = tid; p < nact * kD; p += NT) {       // dWi += vislet^T @ dVe
      const int n = p >> 4, d = p & 15;
      racc[go.wi + p] += fmaf(sVis[n], sdVe[d], sVis[NP1 + n] * sdVe[kD + d]);
    }
    __syncthreads();
  }
  float* row = a.part + ((size_t)s * a.ngroup + grp) * (size_t)P2;
  for (int p = tid; p < P2; p += NT) row[p] = racc[p];
  STAMP(32);
}

// pass 1: slice k sums rows k, k + kGradSlices, ... (fixed order)
__global__ void __launch_bounds__(256) g2k_grad_reduce1_kernel(const float* __restrict__ part,
                                                               float* __restrict__ red, int rows,
                                                               int width) {
  const int p = blockIdx.x * 256 + threadIdx.x, k = blockIdx.y;
  if (p >= width) return;
  float acc = 0.f;
#pragma unroll 16
  for (int r = k; r < rows; r += kGradSlices) acc += part[(size_t)r * width + p];   // loads in flight
  red[(size_t)k * width + p] = acc;
}

// pass 2: the slices in order
__global__ void __launch_bounds__(256) g2k_grad_reduce2_kernel(const float* __restrict__ red,
                                                               float* __restrict__ grad, int width) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= width) return;
  float v[kGradSlices];                             // every slice's load in flight at once
#pragma unroll
  for (int k = 0; k < kGradSlices; ++k) v[k] = red[(size_t)k * width + p];
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < kGradSlices; ++k) acc += v[k];
  grad[p] = acc;
}

// Optimizer step (argParser.py:38-47: grad_clip, learning_rate, decay_rate):
// g = grad / count, clipped by global norm (g * clip / max(||g||, clip)),
// then RMSProp (ms = decay ms + (1 - decay) g^2; p -= lr g / sqrt(ms +
// 1e-10), TF RMSPropOptimizer without momentum) or SGD (ms NULL).  One
// workgroup: the norm is a fixed-order block reduction.
__device__ __forceinline__ void update_apply(float* __restrict__ params, float* __restrict__ ms,
                                             const float* __restrict__ grad, int n, float lr,
                                             float decay, float clip) {
  __shared__ float red[16];
  const int tid = threadIdx.x;
  // up to kPre entries per thread: parameters and mean squares are loaded
  // together with the gradient, before the norm's reduction
  constexpr int kPre = 8;
  const bool pre = n <= kPre * 1024;
  float pg[kPre], pp[kPre], pm[kPre];
  if (pre) {
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int i = tid + j * 1024;
      pg[j] = i < n ? grad[i] : 0.f;
      pp[j] = i < n ? params[i] : 0.f;
      pm[j] = (ms && i < n) ? ms[i] : 0.f;
    }
  }
  const float inv = 1.0f / fmaxf(grad[n + 1], 1.0f);
  float ss = 0.f;
  if (pre) {
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const float g = pg[j] * inv;
      ss = fmaf(g, g, ss);
    }
  } else {
    for (int i = tid; i < n; i += 1024) {
      const float g = grad[i] * inv;
      ss = fmaf(g, g, ss);
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w = 0; w < 16; ++w) tot += red[w];
  const float nrm = sqrtf(tot);
  const float scale = clip > 0.f ? inv * (clip / fmaxf(nrm, clip)) : inv;
  if (pre) {
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int i = tid + j * 1024;
      if (i >= n) break;
      const float g = pg[j] * scale;
      if (ms) {
        const float m = fmaf(decay, pm[j], (1.f - decay) * g * g);
        ms[i] = m;
        params[i] = pp[j] - lr * g / sqrtf(m + 1e-10f);
      } else {
        params[i] = fmaf(-lr, g, pp[j]);
      }
    }
    return;
  }
  for (int i = tid; i < n; i += 1024) {
    const float g = grad[i] * scale;
    if (ms) {
      const float m = fmaf(decay, ms[i], (1.f - decay) * g * g);
      ms[i] = m;
      params[i] -= lr * g / sqrtf(m + 1e-10f);
    } else {
      params[i] = fmaf(-lr, g, params[i]);
    }
  }
}

__global__ void __launch_bounds__(1024) g2k_update_kernel(float* __restrict__ params,
                                                          float* __restrict__ ms,
                                                          const float* __restrict__ grad, int n,
                                                          float lr, float decay, float clip) {
  update_apply(params, ms, grad, n, lr, decay, clip);
}

// one rank (nothing to all-reduce): the second reduction pass and the update
// in one workgroup — the same slice sums as g2k_grad_reduce2_kernel (grad is
// still written), then the same update as g2k_update_kernel
__global__ void __launch_bounds__(1024) g2k_reduce2_update_kernel(const float* __restrict__ slices,
                                                                  float* __restrict__ grad, int width,
                                                                  float* __restrict__ params,
                                                                  float* __restrict__ ms, int n,
                                                                  float lr, float decay, float clip) {
  for (int p = threadIdx.x; p < width; p += 1024) {
    float v[kGradSlices];
#pragma unroll
    for (int k = 0; k < kGradSlices; ++k) v[k] = slices[(size_t)k * width + p];
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < kGradSlices; ++k) acc += v[k];
    grad[p] = acc;
  }
  __syncthreads();   // the workgroup's grad stores are visible to the whole workgroup
  update_apply(params, ms, grad, n, lr, decay, clip);
}

// ---------------------------------------------------------------------------
// a5 static-context input (train.py:92-113, 154-158):
//   _2dconv = lambda * conv2d_VALID(pad(img, [[1,1],[0,1],[0,0]]), K)  [D, D]
//   G       = _2dconv @ stat_mask,  stat_mask[j][t] = t / T           [D, T]
// (tf.nn.conv2d is a cross-correlation; K is the reference's
// [H+3-D, W+2-D, C, 1] filter, so the VALID output is D x D.)  One-off work
// (~3e8 MACs for a 576x720 image): g2k_ctx_conv_kernel takes one filter row
// a per workgroup, stages it and the D padded image rows it meets in LDS and
// forms every output's partial over that row; g2k_ctx_reduce_kernel sums the
// partials over a in a fixed order (deterministic) and forms G.
// ---------------------------------------------------------------------------
struct CtxArgs {
  const float* img;
  const float* filt;
  float* part;      // [KH][D * D]
  float* out;       // [D, D] or NULL
  float* G;         // [D, T] or NULL
  int Hh, Ww, C, D, KH, KW;
  float lambda;
};

__global__ void __launch_bounds__(256) g2k_ctx_conv_kernel(CtxArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int C = a.C, D = a.D, KW = a.KW, pitch = (a.Ww + 1) * C;   // padded row: Ww + 1 columns
  float* sK = smem;                                                // filter row `row` [KW][C]
  float* sI = smem + ((KW * C + 3) & ~3);                          // padded rows row .. row+D-1
  for (int i = tid; i < KW * C; i += 256) sK[i] = a.filt[(size_t)row * KW * C + i];
  for (int i = tid; i < D * pitch; i += 256) {
    const int r = i / pitch, x = i - r * pitch;
    const int pr = row + r;                                        // padded row index
    const bool in = pr >= 1 && pr <= a.Hh && x < a.Ww * C;
    sI[i] = in ? a.img[(size_t)(pr - 1) * a.Ww * C + x] : 0.f;
  }
  __syncthreads();
  if (tid < D * D) {
    const int i = tid / D, j = tid - (tid / D) * D;
    const float* src = sI + i * pitch + j * C;
    const int n = KW * C;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int k = 0;
    for (; k + 4 <= n; k += 4) {
      a0 = fmaf(src[k], sK[k], a0);
      a1 = fmaf(src[k + 1], sK[k + 1], a1);
      a2 = fmaf(src[k + 2], sK[k + 2], a2);
      a3 = fmaf(src[k + 3], sK[k + 3], a3);
    }
    for (; k < n; ++k) a0 = fmaf(src[k], sK[k], a0);
    a.part[(size_t)row * D * D + tid] = (a0 + a1) + (a2 + a3);
  }
}

// one workgroup per output row i: slice s of 256 / D threads sums filter rows
// a = s, s + slices, ... for column j; then the slices in order, lambda, G
__global__ void __launch_bounds__(256) g2k_ctx_reduce_kernel(CtxArgs a) {
  __shared__ float red[256];
  __shared__ float rowv[32];
  const int i = blockIdx.x, tid = threadIdx.x, D = a.D;
  const int slices = 256 / D, j = tid % D, sl = tid / D;
  float acc = 0.f;
  if (sl < slices) {
#pragma unroll 4
    for (int r = sl; r < a.KH; r += slices) acc += a.part[(size_t)r * D * D + i * D + j];
  }
  red[tid] = acc;
  __syncthreads();
  if (tid < D) {
    float v = 0.f;
    for (int s = 0; s < slices; ++s) v += red[s * D + tid];
    v *= a.lambda;
    rowv[tid] = v;
    if (a.out) a.out[i * D + tid] = v;
  }
  __syncthreads();
  if (a.G && tid < kT) {
    float rs = 0.f;
    for (int q = 0; q < D; ++q) rs += rowv[q];
    a.G[i * kT + tid] = rs * ((float)tid / (float)kT);
  }
}

// ---------------------------------------------------------------------------
// host-side validation / geometry
// ---------------------------------------------------------------------------
int validate_common(const g2k_dims* d, bool need_F) {
  if (!d) return set_err(G2K_EINVAL, "dims is NULL");
  if (d->T != kT || d->L != kL || d->D != kD)
    return set_err(G2K_EUNSUPPORTED, "unsupported geometry T=%d L=%d D=%d (need 8/12/16)", d->T,
                   d->L, d->D);
  if (d->S < 0) return set_err(G2K_EINVAL, "S=%d < 0", d->S);
  if (d->Nmax < 1 || d->Nmax > kMaxN)
    return set_err(G2K_EINVAL, "Nmax=%d outside [1, %d]", d->Nmax, kMaxN);
  if (need_F && d->F < 0) return set_err(G2K_EINVAL, "F=%d < 0", d->F);
  return G2K_OK;
}

int validate_weights(const g2k_weights* w, bool need_embed) {
  if (!w) return set_err(G2K_EINVAL, "weights is NULL");
  if (!w->Wv || !w->bv || !w->Wr || !w->Wc || !w->Wo)
    return set_err(G2K_EINVAL, "a model weight pointer is NULL");
  if (need_embed && (!w->Wi || !w->Wii)) return set_err(G2K_EINVAL, "Wi/Wii is NULL");
  return G2K_OK;
}

struct StepPlan {
  int nchunk;
  int64_t lds_bytes, ws_bytes;
};

StepPlan plan_step(const g2k_dims* d) {
  StepPlan p = {0, 0, 0};
  const int F = d->F < 1 ? 1 : d->F;
  p.nchunk = (F + kFramesPerWG - 1) / kFramesPerWG;
  p.lds_bytes = (int64_t)frame_layout(d->Nmax, d->stride).total * 4;
  const int64_t as_bytes = (int64_t)d->S * (d->F > 0 ? d->F : 0) * kD * kD * 4;
  p.ws_bytes = as_bytes + (int64_t)d->S * p.nchunk * 8 * 4;
  return p;
}

// Waves per recurrence workgroup: 4 (one per SIMD).  8 waves (two per SIMD)
// measured 0-5 % slower at H = 128 / 256 (tools/tune_recur.py); kept as a
// tuning option.
int recur_waves(int H) {
  const char* env = getenv("G2K_RECUR_WAVES");   // tuning override (4 or 8)
  if (env && (atoi(env) == 4 || (atoi(env) == 8 && H >= 128))) return atoi(env);
  return 4;
}

int launch_recur(const RecurArgs& r, int S, hipStream_t st) {
  const int nw = recur_waves(r.H);
  const int tpw = r.H / (16 * nw);
  dim3 g(S);
  if (nw == 4) {
    switch (tpw) {
      case 1: hipLaunchKernelGGL((g2k_recur_kernel<1, 4>), g, dim3(256), 0, st, r); break;
      case 2: hipLaunchKernelGGL((g2k_recur_kernel<2, 4>), g, dim3(256), 0, st, r); break;
      case 4: hipLaunchKernelGGL((g2k_recur_kernel<4, 4>), g, dim3(256), 0, st, r); break;
      case 8: hipLaunchKernelGGL((g2k_recur_kernel<8, 4>), g, dim3(256), 0, st, r); break;
      default: return set_err(G2K_EUNSUPPORTED, "H=%d unsupported", r.H);
    }
  } else {
    switch (tpw) {
      case 1: hipLaunchKernelGGL((g2k_recur_kernel<1, 8>), g, dim3(512), 0, st, r); break;
      case 2: hipLaunchKernelGGL((g2k_recur_kernel<2, 8>), g, dim3(512), 0, st, r); break;
      case 4: hipLaunchKernelGGL((g2k_recur_kernel<4, 8>), g, dim3(512), 0, st, r); break;
      default: return set_err(G2K_EUNSUPPORTED, "H=%d unsupported", r.H);
    }
  }
  return G2K_OK;
}

// Fused scene kernel geometry: producer waves (NP).  Measured (gpurun_out
// d38, 400 steps): eth_hotel_synth (H 128, Nmax 32) NP 8 19.9 us vs NP 12
// 20.2, NP 6 22.2, NP 4 24.3; H 256 / Nmax 64: NP 12 28.2 vs NP 8 29.6;
// dense crowd (H 256, Nmax 256): NP 12 53.2 vs NP 8 60.5; k-fold (H 128,
// Nmax 64, d39): NP 12 23.6 vs NP 8 25.4.  So 12 producers (16 waves, 4 per
// SIMD) once H >= 256 or Nmax >= 64, else 8.
// G2K_SCENE_NP in {4, 6, 8, 12} is a tuning override.
int scene_producers(int H, int Nmax) {
  int np = (H >= 256 || Nmax >= 64) ? 12 : 8;
  const char* env = getenv("G2K_SCENE_NP");
  if (env && (atoi(env) == 4 || atoi(env) == 6 || atoi(env) == 8 || atoi(env) == 12)) np = atoi(env);
  if (H >= 512) np = 4;            // TPW 8 needs > 128 VGPRs: at most 512 threads
  return np;
}

SceneLayout scene_layout(const g2k_dims* d, int NP) {
  int fc = d->F < 1 ? 1 : (d->F < kSceneChunk ? d->F : kSceneChunk);
  SceneLayout l = scene_layout_fc(d->Nmax, d->stride, fc, NP);
  while ((int64_t)l.total * 4 > 160 * 1024 && fc > 1) {
    fc = (fc + 1) / 2;
    l = scene_layout_fc(d->Nmax, d->stride, fc, NP);
  }
  return l;
}

bool use_split_step() {
  const char* env = getenv("G2K_STEP_SPLIT");   // A/B switch: the two-kernel step
  return env && atoi(env) == 1;
}

// One scene-kernel launch; MODE = options | kModeDma16 selects the
// instantiation.  Every (TPW, NP) has the default-option modes; the bench
// geometry (TPW 2, NP 8) has all option modes for A/B runs.
template <int TPW, int NP, int MODE>
void launch_scene_k(const StepArgs& a, const SceneLayout& l, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((g2k_scene_kernel<TPW, NP, MODE>), dim3(a.d.S), dim3(64 * (kRecW + NP)), lds, st,
                     a, l);
}

template <int TPW, int NP>
int launch_scene_mode(const StepArgs& a, const SceneLayout& l, size_t lds, hipStream_t st) {
  const int mode = a.opts | (a.dma16 ? kModeDma16 : 0);
  constexpr int kD0 = kSceneOptsDefault, kD1 = kSceneOptsDefault | kModeDma16;
  if (mode == kD0) { launch_scene_k<TPW, NP, kD0>(a, l, lds, st); return G2K_OK; }
  if (mode == kD1) { launch_scene_k<TPW, NP, kD1>(a, l, lds, st); return G2K_OK; }
  if constexpr (TPW == 2 && NP == 8) {
    switch (mode) {
      case 0: launch_scene_k<2, 8, 0>(a, l, lds, st); return G2K_OK;
      case 1: launch_scene_k<2, 8, 1>(a, l, lds, st); return G2K_OK;
      case 2: launch_scene_k<2, 8, 2>(a, l, lds, st); return G2K_OK;
      case 3: launch_scene_k<2, 8, 3>(a, l, lds, st); return G2K_OK;
      case 4: launch_scene_k<2, 8, 4>(a, l, lds, st); return G2K_OK;
      case 5: launch_scene_k<2, 8, 5>(a, l, lds, st); return G2K_OK;
      case 6: launch_scene_k<2, 8, 6>(a, l, lds, st); return G2K_OK;
      case 7: launch_scene_k<2, 8, 7>(a, l, lds, st); return G2K_OK;
      default: break;
    }
  }
  return set_err(G2K_EUNSUPPORTED, "scene options %d not built for H=%d, NP=%d", a.opts, a.d.H, NP);
}

template <int NP>
int launch_scene_np(const StepArgs& a, const SceneLayout& l, hipStream_t st) {
  size_t lds = (size_t)l.total * 4;
  if (const char* e = getenv("G2K_LDS_MIN_KB")) {   // tuning: occupancy experiments
    const size_t m = (size_t)atoi(e) * 1024;
    if (m > lds && m <= 160 * 1024) lds = m;
  }
  switch (a.d.H / 64) {
    case 1: return launch_scene_mode<1, NP>(a, l, lds, st);
    case 2: return launch_scene_mode<2, NP>(a, l, lds, st);
    case 4: return launch_scene_mode<4, NP>(a, l, lds, st);
    default: return set_err(G2K_EUNSUPPORTED, "H=%d unsupported with %d producer waves", a.d.H, NP);
  }
}

int launch_scene(const StepArgs& a, const SceneLayout& l, int NP, hipStream_t st) {
  if (a.d.H == 512) return launch_scene_mode<8, 4>(a, l, (size_t)l.total * 4, st);
  switch (NP) {
    case 4: return launch_scene_np<4>(a, l, st);
    case 6: return launch_scene_np<6>(a, l, st);
    case 8: return launch_scene_np<8>(a, l, st);
    case 12: return launch_scene_np<12>(a, l, st);
    default: return set_err(G2K_EUNSUPPORTED, "NP=%d", NP);
  }
}

int validate_H(int H) {
  if (H < 64 || H > 512 || (H % 64) || (H / 64) == 3 || (H / 64) == 5 || (H / 64) == 6 ||
      (H / 64) == 7)
    return set_err(G2K_EUNSUPPORTED, "H=%d must be 64, 128, 256 or 512", H);
  return G2K_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int g2k_abi_version(void) { return G2K_ABI_VERSION; }

const char* g2k_last_error(void) { return g_err; }

#ifdef G2K_STAMPS_SCENE
int g2k_debug_sstamps(unsigned* host) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g2k_sstamps), 4 * 128 * sizeof(unsigned));
}
#endif
#ifdef G2K_STAMPS
int g2k_debug_stamps(unsigned long long* host, int n) {
  if (n > 64) n = 64;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g2k_stamps), n * sizeof(unsigned long long));
}
#endif

int64_t g2k_step_lds_bytes(const g2k_dims* d) {
  if (validate_common(d, true) != G2K_OK) return 0;
  return plan_step(d).lds_bytes;
}

int64_t g2k_step_workspace_bytes(const g2k_dims* d) {
  if (validate_common(d, true) != G2K_OK) return -1;
  return plan_step(d).ws_bytes;
}

int g2k_step_fused_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                       const float* vislet, const float* G, const float* targets,
                       const int32_t* n_active, const int32_t* n_frames,
                       const uint8_t* ped_mask, const float* h_in, float* h_out, float* pred,
                       float* metrics, float* A_out, float* cost_out, float lambda,
                       void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = validate_common(d, true);
  if (rc) return rc;
  if ((rc = validate_weights(w, true))) return rc;
  if ((rc = validate_H(d->H))) return rc;
  if (d->stride < 0) return set_err(G2K_EINVAL, "stride=%d < 0", d->stride);
  if (d->F > 0 && d->W < (d->F - 1) * d->stride + kT)
    return set_err(G2K_EINVAL, "W=%d < (F-1)*stride + T = %d", d->W, (d->F - 1) * d->stride + kT);
  if (!pos || !vislet || !G || !targets || !n_active || !h_in || !h_out || !pred || !metrics)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!aligned16(targets) || !aligned16(workspace) || !aligned16(h_in) || !aligned16(h_out))
    return set_err(G2K_EINVAL, "targets, h_in, h_out and workspace must be 16-byte aligned");
  if (((uintptr_t)pos & 7u) != 0) return set_err(G2K_EINVAL, "pos must be 8-byte aligned");
  if (d->S == 0) return G2K_OK;
  const StepPlan p = plan_step(d);
  if (p.lds_bytes > 160 * 1024)
    return set_err(G2K_ELDS, "Nmax=%d, stride=%d needs %lld bytes of LDS", d->Nmax, d->stride,
                   (long long)p.lds_bytes);
  if (!workspace || workspace_bytes < p.ws_bytes)
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed (got %lld)", (long long)p.ws_bytes,
                   (long long)workspace_bytes);
  StepArgs a;
  a.d = *d; a.w = *w; a.pos = pos; a.vislet = vislet; a.G = G; a.targets = targets;
  a.n_active = n_active; a.n_frames = n_frames; a.ped_mask = ped_mask; a.h_in = h_in;
  a.h_out = h_out; a.pred = pred; a.metrics = metrics; a.A_out = A_out; a.cost_out = cost_out;
  a.lambda = lambda; a.nchunk = p.nchunk;
  a.dma16 = (d->Nmax % 2 == 0) && aligned16(pos) && aligned16(vislet) && aligned16(G) &&
            aligned16(w->Wi) && aligned16(w->Wo) && aligned16(w->Wii) && aligned16(w->Wv) &&
            aligned16(w->bv) && aligned16(w->Wr) && aligned16(w->Wc);
  // 16-byte staging measured 0.6 us per step SLOWER than the 4-byte LDS-DMA
  // at eth_hotel_synth (gpurun_out d30: 20.3 vs 19.6 us), so it is opt-in
  if (const char* e = getenv("G2K_DMA16")) { if (atoi(e) != 1) a.dma16 = 0; } else a.dma16 = 0;
  a.opts = kSceneOptsDefault;
  if (const char* e = getenv("G2K_SCENE_OPTS")) a.opts = atoi(e) & 3;          // A/B switch
  a.ws_as = static_cast<float*>(workspace);
  a.ws_part = a.ws_as + (size_t)d->S * d->F * kD * kD;
  hipStream_t st = (hipStream_t)stream;
  if (!use_split_step()) {
    const int NP = scene_producers(d->H, d->Nmax);
    const SceneLayout l = scene_layout(d, NP);
    if ((int64_t)l.total * 4 > 160 * 1024)
      return set_err(G2K_ELDS, "Nmax=%d, stride=%d needs %lld bytes of LDS", d->Nmax, d->stride,
                     (long long)l.total * 4);
    if ((rc = launch_scene(a, l, NP, st))) return rc;
    return check_launch("g2k_step_fused_f32/scene");
  }
  if (d->F > 0) {
    hipLaunchKernelGGL(g2k_frames_kernel, dim3(p.nchunk, d->S), dim3(kNT), p.lds_bytes, st, a);
    if ((rc = check_launch("g2k_step_fused_f32/frames"))) return rc;
  }
  RecurArgs r;
  r.att = a.ws_as; r.h_in = h_in; r.h_out = h_out; r.n_frames = n_frames;
  r.ws_part = a.ws_part; r.metrics = metrics; r.F = d->F; r.H = d->H;
  r.nchunk = d->F > 0 ? p.nchunk : 0; r.raw_attn = 0;
  if ((rc = launch_recur(r, d->S, st))) return rc;
  return check_launch("g2k_step_fused_f32/recur");
}

int g2k_mcr_forward_f32(const g2k_dims* d, const g2k_weights* w, const float* X,
                        const float* Rel, const float* G, const int32_t* n_active, float* A_out,
                        float* cost_out, float* pred, float lambda, void* stream) {
  int rc = validate_common(d, false);
  if (rc) return rc;
  if ((rc = validate_weights(w, false))) return rc;
  if (!X || !Rel || !G || !n_active || !A_out || !cost_out || !pred)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (d->S == 0) return G2K_OK;
  FwdArgs a;
  a.d = *d; a.w = *w; a.X = X; a.Rel = Rel; a.G = G; a.n_active = n_active; a.A_out = A_out;
  a.cost_out = cost_out; a.pred = pred; a.lambda = lambda;
  hipLaunchKernelGGL(g2k_mcr_forward_kernel, dim3(d->S), dim3(kNT), 0, (hipStream_t)stream, a);
  return check_launch("g2k_mcr_forward_f32");
}

int g2k_frame_recurrence_f32(const g2k_dims* d, const float* A, float* h, int32_t frames,
                             void* stream) {
  if (!d) return set_err(G2K_EINVAL, "dims is NULL");
  if (d->D != kD) return set_err(G2K_EUNSUPPORTED, "D=%d (need 16)", d->D);
  int rc = validate_H(d->H);
  if (rc) return rc;
  if (!A || !h) return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!aligned16(A) || !aligned16(h)) return set_err(G2K_EINVAL, "A and h must be 16-byte aligned");
  if (frames < 0 || d->S < 0) return set_err(G2K_EINVAL, "negative frames or S");
  if (d->S == 0) return G2K_OK;
  RecurArgs r;
  r.att = A; r.h_in = h; r.h_out = h; r.n_frames = nullptr; r.ws_part = nullptr;
  r.metrics = nullptr; r.F = frames; r.H = d->H; r.nchunk = 0; r.raw_attn = 1;
  if ((rc = launch_recur(r, d->S, (hipStream_t)stream))) return rc;
  return check_launch("g2k_frame_recurrence_f32");
}

int g2k_ade_fde_f32(const g2k_dims* d, const float* pred, const float* targets,
                    const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                    int32_t variant, float* out, void* stream) {
  int rc = validate_common(d, true);
  if (rc) return rc;
  if (!pred || !targets || !n_active || !out)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!aligned16(targets)) return set_err(G2K_EINVAL, "targets must be 16-byte aligned");
  if (d->S == 0) return G2K_OK;
  ErrArgs a;
  a.d = *d; a.pred = pred; a.targets = targets; a.n_active = n_active; a.n_frames = n_frames;
  a.ped_mask = ped_mask; a.out = out;
  hipStream_t st = (hipStream_t)stream;
  if (variant == 0) {
    hipLaunchKernelGGL(g2k_errors_v0_kernel, dim3(d->S), dim3(kNT), 0, st, a);
  } else if (variant == 1) {
    hipLaunchKernelGGL(g2k_errors_v1_kernel, dim3(d->S), dim3(64), 0, st, a);
  } else {
    return set_err(G2K_EINVAL, "unknown error variant %d", variant);
  }
  return check_launch("g2k_ade_fde_f32");
}

int g2k_infer_rlns_f32(const float* adj, float* out, int64_t rows, int32_t cols, void* stream) {
  if (!adj || !out || rows < 0 || cols < 0) return set_err(G2K_EINVAL, "bad arguments");
  const int64_t n = rows * (int64_t)cols;
  if (n == 0) return G2K_OK;
  hipLaunchKernelGGL(g2k_sigmoid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, adj, out, n);
  return check_launch("g2k_infer_rlns_f32");
}

int g2k_eval_rln_ngh_f32(const float* adj, float* out, int64_t rows, int32_t cols, void* stream) {
  if (!adj || !out || rows < 0 || cols < 1) return set_err(G2K_EINVAL, "bad arguments");
  if (rows == 0) return G2K_OK;
  hipLaunchKernelGGL(g2k_row_softmax_kernel, dim3((unsigned)rows), dim3(64), 0,
                     (hipStream_t)stream, adj, out, cols);
  return check_launch("g2k_eval_rln_ngh_f32");
}

int g2k_gridlstm_f32(const float* in, int64_t ld_in, const float* state, int64_t ld_state,
                     const float* W, const float* b, const float* peep, float* out,
                     float* state_out, int64_t rows, int32_t blocks, int32_t feature_size,
                     int32_t num_units, void* stream) {
  if (!in || !state || !W || !b || !out || !state_out)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (rows < 0 || blocks < 1 || feature_size < 1 || num_units < 1)
    return set_err(G2K_EINVAL, "rows=%lld blocks=%d feature_size=%d num_units=%d", (long long)rows,
                   blocks, feature_size, num_units);
  const int64_t w_out = (int64_t)blocks * 2 * num_units;
  if (ld_in < (int64_t)blocks * feature_size || ld_state < w_out)
    return set_err(G2K_EINVAL, "row pitch too small (ld_in=%lld, ld_state=%lld)", (long long)ld_in,
                   (long long)ld_state);
  if (state_out == state && ld_state != w_out)
    return set_err(G2K_EINVAL, "state_out may alias state only when ld_state == blocks*2*num_units");
  const bool ok_u = num_units == 1 || num_units == 2 || num_units == 4;
  const bool ok_f = feature_size == 2 || feature_size == 4 || feature_size == 8;
  if (!ok_u || !ok_f)
    return set_err(G2K_EUNSUPPORTED, "num_units=%d feature_size=%d (built: units 1/2/4, features 2/4/8)",
                   num_units, feature_size);
  if (rows == 0) return G2K_OK;
  GridArgs a;
  a.in = in; a.state = state; a.W = W; a.b = b; a.peep = peep; a.out = out; a.state_out = state_out;
  a.rows = rows; a.ld_in = ld_in; a.ld_state = ld_state; a.K = blocks;
  const dim3 g((unsigned)((rows + 255) / 256)), blk(256);
  hipStream_t st = (hipStream_t)stream;
  const int key = num_units * 16 + feature_size;
  switch (key) {
    case 1 * 16 + 2: hipLaunchKernelGGL((g2k_gridlstm_kernel<1, 2>), g, blk, 0, st, a); break;
    case 1 * 16 + 4: hipLaunchKernelGGL((g2k_gridlstm_kernel<1, 4>), g, blk, 0, st, a); break;
    case 1 * 16 + 8: hipLaunchKernelGGL((g2k_gridlstm_kernel<1, 8>), g, blk, 0, st, a); break;
    case 2 * 16 + 2: hipLaunchKernelGGL((g2k_gridlstm_kernel<2, 2>), g, blk, 0, st, a); break;
    case 2 * 16 + 4: hipLaunchKernelGGL((g2k_gridlstm_kernel<2, 4>), g, blk, 0, st, a); break;
    case 2 * 16 + 8: hipLaunchKernelGGL((g2k_gridlstm_kernel<2, 8>), g, blk, 0, st, a); break;
    case 4 * 16 + 2: hipLaunchKernelGGL((g2k_gridlstm_kernel<4, 2>), g, blk, 0, st, a); break;
    case 4 * 16 + 4: hipLaunchKernelGGL((g2k_gridlstm_kernel<4, 4>), g, blk, 0, st, a); break;
    default:         hipLaunchKernelGGL((g2k_gridlstm_kernel<4, 8>), g, blk, 0, st, a); break;
  }
  return check_launch("g2k_gridlstm_f32");
}

int64_t g2k_grad_size(const g2k_dims* d) {
  if (validate_common(d, false) != G2K_OK) return -1;
  return grad_params(d->Nmax);
}

// launch shape of the gradient: g2k_grad_seq_kernel with `frames` frames per
// workgroup (default), or g2k_grad_kernel with one wave per frame when the
// G2K_GRAD_GW A/B override is set
struct GradLaunch {
  bool seq;
  int frames;   // frames per workgroup
  int ngroup;
};
static GradLaunch grad_launch(const g2k_dims* d) {
  GradLaunch g;
  g.seq = getenv("G2K_GRAD_GW") == nullptr &&
          (size_t)4 * grad_seq_lds_floats(d->Nmax) <= 160 * 1024;
  g.frames = g.seq ? grad_seq_fpg(d) : grad_gw(d->Nmax);
  g.ngroup = (d->F + g.frames - 1) / g.frames;
  return g;
}

int64_t g2k_grad_workspace_bytes(const g2k_dims* d) {
  if (validate_common(d, true) != G2K_OK) return -1;
  const int64_t ngroup = grad_launch(d).ngroup;
  return ((int64_t)d->S * ngroup + kGradSlices) * (grad_params(d->Nmax) + 2) * 4;
}

static int step_grad(const g2k_dims* d, const g2k_weights* w, const float* pos,
                     const float* vislet, const float* G, const float* targets,
                     const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                     float lambda, float* grad, void* workspace, int64_t workspace_bytes,
                     void* stream, float* upd_params, float* upd_ms, float lr, float decay,
                     float grad_clip) {
  int rc = validate_common(d, true);
  if (rc) return rc;
  if ((rc = validate_weights(w, true))) return rc;
  if (d->stride < 0) return set_err(G2K_EINVAL, "stride=%d < 0", d->stride);
  if (d->F > 0 && d->W < (d->F - 1) * d->stride + kT)
    return set_err(G2K_EINVAL, "W=%d < (F-1)*stride + T = %d", d->W, (d->F - 1) * d->stride + kT);
  if (!pos || !vislet || !G || !targets || !n_active || !grad)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (((uintptr_t)pos & 7u) != 0) return set_err(G2K_EINVAL, "pos must be 8-byte aligned");
  const int64_t need = g2k_grad_workspace_bytes(d);
  if (!workspace || workspace_bytes < need)
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed (got %lld)", (long long)need,
                   (long long)workspace_bytes);
  const GradLaunch gl = grad_launch(d);
  const int GW = gl.frames, ngroup = gl.ngroup;
  const int width = grad_params(d->Nmax) + 2;
  hipStream_t st = (hipStream_t)stream;
  if (d->S == 0 || ngroup == 0) {
    if (hipMemsetAsync(grad, 0, (size_t)width * 4, st) != hipSuccess)
      return set_err(G2K_ELAUNCH, "g2k_step_grad_f32: memset failed");
    if (upd_params)
      hipLaunchKernelGGL(g2k_update_kernel, dim3(1), dim3(1024), 0, st, upd_params, upd_ms, grad,
                         width - 2, lr, decay, grad_clip);
    return check_launch("g2k_step_grad_f32/empty");
  }
  const size_t lds = gl.seq ? (size_t)4 * grad_seq_lds_floats(d->Nmax)
                            : (size_t)4 * (grad_shared_floats(d->Nmax) + GW * grad_scratch_floats(d->Nmax));
  if (lds > 160 * 1024) return set_err(G2K_ELDS, "Nmax=%d needs %zu bytes of LDS", d->Nmax, lds);
  GradArgs a;
  a.d = *d; a.w = *w; a.pos = pos; a.vislet = vislet; a.G = G; a.targets = targets;
  a.n_active = n_active; a.n_frames = n_frames; a.ped_mask = ped_mask; a.lambda = lambda;
  a.part = static_cast<float*>(workspace); a.ngroup = ngroup;
  float* red = a.part + (size_t)d->S * ngroup * width;
  const dim3 grid(ngroup, d->S);
  if (gl.seq && (160 * 1024) / lds >= (size_t)kGradSeqWgPerCu)
    hipLaunchKernelGGL((g2k_grad_seq_kernel<kGradSeqWgPerCu>), grid, dim3(256), lds, st, a, GW);
  else if (gl.seq)
    hipLaunchKernelGGL((g2k_grad_seq_kernel<2>), grid, dim3(256), lds, st, a, GW);
  else if (GW == 4)
    hipLaunchKernelGGL((g2k_grad_kernel<4>), grid, dim3(256), lds, st, a);
  else if (GW == 2)
    hipLaunchKernelGGL((g2k_grad_kernel<2>), grid, dim3(128), lds, st, a);
  else
    hipLaunchKernelGGL((g2k_grad_kernel<1>), grid, dim3(64), lds, st, a);
  if ((rc = check_launch("g2k_step_grad_f32/grad"))) return rc;
  const unsigned gx = (unsigned)((width + 255) / 256);
  hipLaunchKernelGGL(g2k_grad_reduce1_kernel, dim3(gx, kGradSlices), dim3(256), 0, st, a.part, red,
                     d->S * ngroup, width);
  if (upd_params)
    hipLaunchKernelGGL(g2k_reduce2_update_kernel, dim3(1), dim3(1024), 0, st, red, grad, width,
                       upd_params, upd_ms, width - 2, lr, decay, grad_clip);
  else
    hipLaunchKernelGGL(g2k_grad_reduce2_kernel, dim3(gx), dim3(256), 0, st, red, grad, width);
  return check_launch("g2k_step_grad_f32/reduce");
}

int g2k_step_grad_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                      const float* vislet, const float* G, const float* targets,
                      const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                      float lambda, float* grad, void* workspace, int64_t workspace_bytes,
                      void* stream) {
  return step_grad(d, w, pos, vislet, G, targets, n_active, n_frames, ped_mask, lambda, grad,
                   workspace, workspace_bytes, stream, nullptr, nullptr, 0.f, 0.f, 0.f);
}

int g2k_step_grad_update_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                             const float* vislet, const float* G, const float* targets,
                             const int32_t* n_active, const int32_t* n_frames,
                             const uint8_t* ped_mask, float lambda, float* grad, void* workspace,
                             int64_t workspace_bytes, float* params, float* ms, float lr,
                             float decay, float grad_clip, void* stream) {
  if (!params) return set_err(G2K_EINVAL, "params is NULL");
  return step_grad(d, w, pos, vislet, G, targets, n_active, n_frames, ped_mask, lambda, grad,
                   workspace, workspace_bytes, stream, params, ms, lr, decay, grad_clip);
}

int g2k_update_f32(float* params, float* ms, const float* grad, int64_t n_params, float lr,
                   float decay, float grad_clip, void* stream) {
  if (!params || !grad || n_params < 0 || n_params > (1 << 30))
    return set_err(G2K_EINVAL, "bad arguments");
  if (n_params == 0) return G2K_OK;
  hipLaunchKernelGGL(g2k_update_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, params, ms, grad,
                     (int)n_params, lr, decay, grad_clip);
  return check_launch("g2k_update_f32");
}

int64_t g2k_context_conv_workspace_bytes(int32_t Hh, int32_t Ww, int32_t D) {
  if (Hh < 1 || Ww < 1 || D < 1 || D > 16 || Hh + 3 - D < 1 || Ww + 2 - D < 1) return -1;
  return (int64_t)(Hh + 3 - D) * D * D * 4;
}

int g2k_context_conv_f32(const float* img, int32_t Hh, int32_t Ww, int32_t C, const float* filt,
                         int32_t D, float lambda, float* out, float* G, void* workspace,
                         int64_t workspace_bytes, void* stream) {
  if (!img || !filt || (!out && !G)) return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (C < 1 || C > 4) return set_err(G2K_EUNSUPPORTED, "C=%d channels (1..4)", C);
  const int64_t need = g2k_context_conv_workspace_bytes(Hh, Ww, D);
  if (need < 0) return set_err(G2K_EINVAL, "image %dx%d, D=%d (D in 1..16, image >= D)", Hh, Ww, D);
  if (!workspace || workspace_bytes < need)
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed", (long long)need);
  CtxArgs a;
  a.img = img; a.filt = filt; a.part = static_cast<float*>(workspace); a.out = out; a.G = G;
  a.Hh = Hh; a.Ww = Ww; a.C = C; a.D = D; a.KH = Hh + 3 - D; a.KW = Ww + 2 - D; a.lambda = lambda;
  const size_t lds = (size_t)4 * (((a.KW * C + 3) & ~3) + (size_t)D * (Ww + 1) * C);
  if (lds > 160 * 1024) return set_err(G2K_ELDS, "image width %d needs %zu bytes of LDS", Ww, lds);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(g2k_ctx_conv_kernel, dim3(a.KH), dim3(256), lds, st, a);
  hipLaunchKernelGGL(g2k_ctx_reduce_kernel, dim3(D), dim3(256), 0, st, a);
  return check_launch("g2k_context_conv_f32");
}

}  // extern "C"
