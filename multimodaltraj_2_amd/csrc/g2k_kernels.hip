// g2k_kernels.hip — gfx950 (CDNA4) kernels + C ABI for the g2k_lstm_mcr
// per-frame path of serenetech90/multimodaltraj_2.
//
// The step (train.py:197-276 over S scenes x F frames) is two launches on one
// stream:
//   1. g2k_frames_kernel — frame-parallel part (a2-a7, a9): grid =
//      (frame chunks) x S, 256 threads.  The chunk's targets arrive in LDS by
//      LDS-DMA (global_load_lds_dwordx4) while the window norms, embeddings,
//      g2k_lstm_mcr forward (X0, E, A, cost, Wc@cost) run as batched tiny
//      matmuls out of LDS; predictions are stored, ADE/FDE partial sums and
//      the attention weights As = softmax(exp(A)/cumsum(exp(A))) go to a
//      workspace.  Many small workgroups per CU hide the latency chains.
//   2. g2k_recur_kernel — frame-sequential part (a8): one workgroup per
//      scene keeps h [16, H] in registers in the v_mfma_f32_16x16x4_f32 C
//      layout; per frame: one MFMA contraction, one row-softmax reduction
//      (16-lane DPP + ONE 4-wave LDS exchange), no global traffic except the
//      LDS-DMA of the scene's As tiles.
// Deterministic: fixed reduction order, no atomics.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdint.h>

#include "g2k_hip.h"

namespace {

constexpr int kT = 8;     // obs_len
constexpr int kL = 12;    // pred_len
constexpr int kL2 = 24;   // 2 * pred_len rows of temp_path
constexpr int kD = 16;    // hidden_len
constexpr int kNT = 256;  // threads per workgroup
constexpr int kMaxN = 256;
constexpr int kRecurChunk = 32;         // As tiles resident in LDS in g2k_recur_kernel
constexpr int kFramesLdsBudget = 48 * 1024;

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

__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// LDS-DMA: 16 bytes per lane, LDS destination = wave-uniform base + 16*lane.
__device__ __forceinline__ void dma16(const float* gsrc, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

// Copy n4 float4s (contiguous, 16-B aligned) global -> LDS with the whole
// workgroup; the caller waits (vmcnt(0)) and barriers before reading.
__device__ __forceinline__ void dma_copy(const float* g, float* lds, int n4, int wv, int lane) {
  for (int i = wv * 64; i < n4; i += kNT) {
    if (i + lane < n4) dma16(g + (size_t)(i + lane) * 4, lds + i * 4);
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

__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp<0xB1>(v));
  v = fmaxf(v, dpp<0x4E>(v));
  v = fmaxf(v, dpp<0x141>(v));
  v = fmaxf(v, dpp<0x140>(v));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
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

// Sum / max over the four 16-lane rows of a wave (lanes r, r+16, r+32, r+48),
// identical bits in all four lanes: v_permlane32_swap + v_permlane16_swap.
__device__ __forceinline__ float sum_rows4(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

__device__ __forceinline__ float max_rows4(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

// ---------------------------------------------------------------------------
// Hidden recurrence (train.py:243-252), h in registers:
//   h <- softmax(h, -1); h <- As @ h; adj <- softmax(h, -1) @ 1; h <- adj * h
// computed as h'^T = softmax(h)^T @ As^T with v_mfma_f32_16x16x4_f32
// (M = 16 columns of h, N = the 16 rows, K = 16 in four k-steps).  Wave w owns
// columns [w*H/4, (w+1)*H/4) as TPW 16-wide tiles; lane l (r = l & 15,
// q = l >> 4) holds ONE row r: h'[r][16t + 4q + i] in x[t][i].  Row softmax
// sums are therefore a local sum plus a 2-step permlane reduction, and one
// 4-wave LDS exchange per frame.  The next frame's A operand
// (softmax(h)[k][c] with k on the lane group) is a wave-local 16x16
// transpose through LDS (no barrier).
//
// One exchange per frame: each wave publishes per-row P = sum e2 and
// Q = sum h' * e2 (e2 = exp(h')).  Z2 = sum_w P_w, adj = sum_w P_w / Z2 (the
// row sum of the softmax, evaluated from the wave partials), h_next =
// adj * h', and the next softmax's numerators exp(adj * h') = e2 * exp(d h')
// with d = adj - 1: |d| is a few ulp (adj == 1 in exact arithmetic) and h' is
// in [0, 1] (convex combinations of softmax outputs), so exp(d h') =
// 1 + d h' + O(1e-13) and the next row sums are P + d Q.
// ---------------------------------------------------------------------------
constexpr int kTP = 20;            // transpose tile row pitch (floats): conflict-free b32 reads
constexpr int kTTile = kD * kTP;   // 320 floats per 16x16 tile

template <int TPW>
struct Recur {
  float x[TPW][4];   // h (before init) / the last h' (after a step)
  float e[TPW][4];   // numerators of the next softmax(h), row r
  float rz;          // 1 / their row sum
  float adj;         // row scale of the last step: h = adj * h'

  __device__ __forceinline__ void load(const float* __restrict__ hs, int H, int wv, int q, int r) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const float4 v = *reinterpret_cast<const float4*>(hs + r * H + wv * (H / 4) + 16 * t + 4 * q);
      x[t][0] = v.x; x[t][1] = v.y; x[t][2] = v.z; x[t][3] = v.w;
    }
    adj = 1.0f;
  }

  __device__ __forceinline__ void store(float* __restrict__ hs, int H, int wv, int q, int r) const {
#pragma unroll
    for (int t = 0; t < TPW; ++t)
      *reinterpret_cast<float4*>(hs + r * H + wv * (H / 4) + 16 * t + 4 * q) =
          make_float4(adj * x[t][0], adj * x[t][1], adj * x[t][2], adj * x[t][3]);
  }

  // softmax prologue on an arbitrary h (tf.nn.softmax max shift), 2 exchanges
  // through `red` (128 floats used only here).
  __device__ __forceinline__ void init(float* red, int wv, int q, int r) {
    float m = x[0][0];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) m = fmaxf(m, x[t][i]);
    m = max_rows4(m);
    if (q == 0) red[wv * 16 + r] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[r], red[16 + r]), fmaxf(red[32 + r], red[48 + r]));
    float p = 0.f;
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        e[t][i] = __expf(x[t][i] - m);
        p += e[t][i];
      }
    p = sum_rows4(p);
    if (q == 0) red[64 + wv * 16 + r] = p;
    __syncthreads();
    rz = rcp((red[64 + r] + red[80 + r]) + (red[96 + r] + red[112 + r]));
  }

  // One frame.  b = As[r][4q..4q+3] of this frame (B operand: As^T[k][r]);
  // as_next = next frame's As tile in LDS (or NULL), its slice is read after
  // the barrier.  sT: this wave's TPW transpose tiles.  red: 128 floats,
  // alternating between two buffers on consecutive frames.
  __device__ __forceinline__ float4 step(const float4 b, const float* as_next, float* sT,
                                         float* red, int wv, int q, int r) {
    // A operand: softmax(h)[k = 4q + ks][c = 16t + r] via a wave-local transpose
#pragma unroll
    for (int t = 0; t < TPW; ++t)
      *reinterpret_cast<float4*>(sT + t * kTTile + r * kTP + 4 * q) =
          make_float4(e[t][0] * rz, e[t][1] * rz, e[t][2] * rz, e[t][3] * rz);
    __builtin_amdgcn_wave_barrier();
    f32x4 acc[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const float* col = sT + t * kTTile + (4 * q) * kTP + r;
      f32x4 c = {0.f, 0.f, 0.f, 0.f};
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(col[0], b.x, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(col[kTP], b.y, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(col[2 * kTP], b.z, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_16x16x4f32(col[3 * kTP], b.w, c, 0, 0, 0);
      acc[t] = c;
    }
    float p = 0.f, qs = 0.f;
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[t][i];
        const float ex = __expf(v);       // h' in [0, 1]: no max shift needed
        x[t][i] = v;
        e[t][i] = ex;
        p += ex;
        qs = fmaf(v, ex, qs);
      }
    p = sum_rows4(p);
    qs = sum_rows4(qs);
    if (q == 0) *reinterpret_cast<float2*>(red + wv * 32 + 2 * r) = make_float2(p, qs);
    __syncthreads();
    float4 nxt = make_float4(0.f, 0.f, 0.f, 0.f);
    if (as_next) nxt = *reinterpret_cast<const float4*>(as_next + r * kD + 4 * q);
    const float2 w0 = *reinterpret_cast<const float2*>(red + 0 * 32 + 2 * r);
    const float2 w1 = *reinterpret_cast<const float2*>(red + 1 * 32 + 2 * r);
    const float2 w2 = *reinterpret_cast<const float2*>(red + 2 * 32 + 2 * r);
    const float2 w3 = *reinterpret_cast<const float2*>(red + 3 * 32 + 2 * r);
    const float r2 = rcp((w0.x + w1.x) + (w2.x + w3.x));
    adj = (w0.x * r2 + w1.x * r2) + (w2.x * r2 + w3.x * r2);
    const float d = adj - 1.0f;
    rz = rcp((fmaf(d, w0.y, w0.x) + fmaf(d, w1.y, w1.x)) + (fmaf(d, w2.y, w2.x) + fmaf(d, w3.y, w3.x)));
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) e[t][i] = fmaf(e[t][i] * d, x[t][i], e[t][i]);
    return nxt;
  }
};

// ---------------------------------------------------------------------------
// Kernel 1: frame-parallel part.  LDS carve (floats; offsets multiple of 4).
// ---------------------------------------------------------------------------
struct FrameLayout {
  int np;   // padded norm row stride
  int o_tgt, o_wi, o_wo, o_nrm, o_v, o_small, o_xa, o_e, o_c, o_m, o_met;
  int total;
};

__host__ __device__ inline int rup4(int x) { return (x + 3) & ~3; }

__host__ __device__ inline FrameLayout frame_layout(int Nmax, int stride, int fa) {
  FrameLayout s;
  const int wc = (fa - 1) * stride + kT;
  s.np = Nmax + 1;
  int o = 0;
  s.o_tgt = o;   o += fa * Nmax * kL2;     // LDS-DMA destination
  s.o_wi = o;    o += rup4(Nmax * kD);
  s.o_wo = o;    o += rup4(kT * Nmax);
  s.o_nrm = o;   o += rup4((wc + 2) * s.np);
  s.o_v = o;     o += rup4((wc + 2) * kD);
  s.o_small = o; o += 1024;
  s.o_xa = o;    o += fa * kD * kD;        // X0, then A / As
  s.o_e = o;     o += fa * kT * kD;        // E
  s.o_c = o;     o += fa * kT * kT;        // cost
  s.o_m = o;     o += fa * kL2 * kT;       // Wc @ cost
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
constexpr int SM_RM = 624;    // [8][16]
constexpr int SM_EC = 752;    // [8][16]  Wv[:,16:18] @ Ve
// end 880 <= 1024

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
  int fchunk;
  int nchunk;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__global__ void __launch_bounds__(kNT) g2k_frames_kernel(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int chunk = blockIdx.x, s = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int Nmax = a.d.Nmax, W = a.d.W, F = a.d.F, stride = a.d.stride;
  const int FA = a.fchunk;
  const int nact = clampi(a.n_active[s], 0, Nmax);
  const int nf = a.n_frames ? clampi(a.n_frames[s], 0, F) : F;
  const int f0 = chunk * FA;
  float* part = a.ws_part + ((size_t)s * a.nchunk + chunk) * 8;
  STAMP(0);

  // frames of this chunk beyond n_frames: zero predictions
  {
    const int z0 = f0 > nf ? f0 : nf;
    const int z1 = (f0 + FA) < F ? (f0 + FA) : F;
    for (int i = tid; i < (z1 - z0) * kL2 * Nmax; i += kNT)
      a.pred[((size_t)s * F + z0) * kL2 * Nmax + i] = 0.f;
  }
  if (f0 >= nf) {                       // uniform per workgroup
    if (tid < 8) part[tid] = 0.f;
    return;
  }
  const int fa = (nf - f0) < FA ? (nf - f0) : FA;
  const int r0 = f0 * stride, wc = (fa - 1) * stride + kT;
  const FrameLayout lay = frame_layout(Nmax, stride, FA);
  float* sTgt = smem + lay.o_tgt;
  float* sWi = smem + lay.o_wi;
  float* sWo = smem + lay.o_wo;
  float* sNrm = smem + lay.o_nrm;
  float* sV = smem + lay.o_v;
  float* sm = smem + lay.o_small;
  float* sXA = smem + lay.o_xa;
  float* sE = smem + lay.o_e;
  float* sC = smem + lay.o_c;
  float* sM = smem + lay.o_m;
  float* sMet = smem + lay.o_met;
  const int np = lay.np;

  // ---- stage 0: targets by LDS-DMA; weights, vislet, window norms --------
  dma_copy(a.targets + ((size_t)s * F + f0) * Nmax * kL2, sTgt, fa * Nmax * (kL2 / 4), wv, lane);
  for (int i = tid; i < Nmax * kD; i += kNT) sWi[i] = (i / kD) < nact ? a.w.Wi[i] : 0.f;
  for (int i = tid; i < kT * Nmax; i += kNT) sWo[i] = a.w.Wo[i];
  if (tid < kD * kT) {
    sm[SM_WII + tid] = a.w.Wii[tid];
    sm[SM_G + tid] = a.lambda * a.G[(size_t)s * kD * kT + tid];   // ngh = lambda*ngh (g2k_lstm_mcr.py:102)
  }
  if (tid < kT * (kD + 2)) sm[SM_WV + tid] = a.w.Wv[tid];
  if (tid < kD) sm[SM_BV + tid] = a.w.bv[tid];
  if (tid < kT * 2) sm[SM_WR + tid] = a.w.Wr[tid];
  if (tid < kL2 * kT) sm[SM_WC + tid] = a.w.Wc[tid];
  {
    const float* vis = a.vislet + (size_t)s * 2 * Nmax;
    for (int i = tid; i < 2 * Nmax; i += kNT) {
      const int c = i / Nmax, n = i - c * Nmax;
      sNrm[(wc + c) * np + n] = n < nact ? vis[i] : 0.f;
    }
    const float2* p2 = reinterpret_cast<const float2*>(a.pos) + ((size_t)s * W + r0) * Nmax;
    for (int i = tid; i < wc * Nmax; i += kNT) {
      const int w = i / Nmax, n = i - w * Nmax;
      float v = 0.f;
      if (n < nact) {
        const float2 p = p2[i];
        v = sqrtf(fmaf(p.x, p.x, p.y * p.y));     // ||(x, y)||_2 (train.py:79)
      }
      sNrm[w * np + n] = v;
    }
  }
  __syncthreads();
  STAMP(1);

  // ---- stage 1: V = nrm @ Wi for the chunk's position rows (+ Ve rows) ----
  // frame f's Bv @ Wi (train.py:179) is rows (f-f0)*stride .. +7 of V.
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
  // ---- stage 2: per-scene Rel/Rm and the Ve part of E ---------------------
  if (tid < kT * kD) {
    const int t = tid >> 4, dcol = tid & 15;
    const float ve0 = sV[wc * kD + dcol], ve1 = sV[(wc + 1) * kD + dcol];
    // Rel = Ve * Ve (train.py:194-195); Rm = Wr @ Rel (g2k_lstm_mcr.py:106)
    sm[SM_RM + tid] = fmaf(sm[SM_WR + 2 * t], ve0 * ve0, sm[SM_WR + 2 * t + 1] * (ve1 * ve1));
    sm[SM_EC + tid] = fmaf(sm[SM_WV + t * (kD + 2) + kD], ve0, sm[SM_WV + t * (kD + 2) + kD + 1] * ve1);
  }
  // ---- stage 3: X0_f = Wii @ U_f  (train.py:180) -------------------------
  {
    const int dcol = tid & 15, k = tid >> 4;
    float wii[kT];
#pragma unroll
    for (int t = 0; t < kT; ++t) wii[t] = sm[SM_WII + k * kT + t];
    for (int fl = 0; fl < fa; ++fl) {
      const float* v = sV + (fl * stride) * kD + dcol;
      float x = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) x = fmaf(wii[t], v[t * kD], x);
      sXA[fl * kD * kD + k * kD + dcol] = x;
    }
  }
  __syncthreads();
  STAMP(2);
  // ---- stage 4: E_f = Wv @ [X0_f; Ve] + bv  (g2k_lstm_mcr.py:105,112) ------
  {
    const int dcol = tid & 15, t = (tid >> 4) & 7;
    float wv16[kD];
#pragma unroll
    for (int k = 0; k < kD; ++k) wv16[k] = sm[SM_WV + t * (kD + 2) + k];
    const float ec = sm[SM_EC + t * kD + dcol];
    const float bvv = sm[SM_BV + dcol];
    for (int fl = tid >> 7; fl < fa; fl += 2) {
      const float* x0 = sXA + fl * kD * kD + dcol;
      float e = 0.f;
#pragma unroll
      for (int k = 0; k < kD; ++k) e = fmaf(wv16[k], x0[k * kD], e);
      sE[fl * kT * kD + t * kD + dcol] = (e + ec) + bvv;
    }
  }
  __syncthreads();
  STAMP(3);
  // ---- stage 5: A_f = g @ (E_f * Rm), cost_f = E_f @ g  (:105-106, :112) ---
  {
    const int dcol = tid & 15, r = tid >> 4;
    float gr[kT], rm[kT];
#pragma unroll
    for (int t = 0; t < kT; ++t) { gr[t] = sm[SM_G + r * kT + t]; rm[t] = sm[SM_RM + t * kD + dcol]; }
    for (int fl = 0; fl < fa; ++fl) {
      const float* e = sE + fl * kT * kD + dcol;
      float x = 0.f;
#pragma unroll
      for (int t = 0; t < kT; ++t) x = fmaf(gr[t], e[t * kD] * rm[t], x);
      sXA[fl * kD * kD + r * kD + dcol] = x;
      if (a.A_out) a.A_out[(((size_t)s * F + f0 + fl) * kD + r) * kD + dcol] = x;
    }
    const int t2 = tid & 7, t1 = (tid >> 3) & 7;
    float gc[kD];
#pragma unroll
    for (int k = 0; k < kD; ++k) gc[k] = sm[SM_G + k * kT + t2];
    for (int fl = tid >> 6; fl < fa; fl += 4) {
      const float* e = sE + fl * kT * kD + t1 * kD;
      float x = 0.f;
#pragma unroll
      for (int k = 0; k < kD; ++k) x = fmaf(e[k], gc[k], x);
      sC[fl * kT * kT + t1 * kT + t2] = x;
      if (a.cost_out) a.cost_out[(((size_t)s * F + f0 + fl) * kT + t1) * kT + t2] = x;
    }
  }
  __syncthreads();
  STAMP(4);
  // ---- stage 6: attention column pass; M_f = Wc @ cost_f (:122) ------------
  for (int task = tid; task < fa * kD; task += kNT)
    attn_column_pass(sXA + (task >> 4) * kD * kD, task & 15);
  for (int task = tid; task < fa * kL2 * kT; task += kNT) {
    const int fl = task / (kL2 * kT), rem = task - fl * kL2 * kT;
    const int jr = rem >> 3, t2 = rem & 7;
    const float* c = sC + fl * kT * kT + t2;
    float x = 0.f;
#pragma unroll
    for (int t = 0; t < kT; ++t) x = fmaf(sm[SM_WC + jr * kT + t], c[t * kT], x);
    sM[fl * kL2 * kT + rem] = x;
  }
  // the DMA'd targets are read in stage 7
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  STAMP(5);
  // ---- stage 7: attention row softmax -> workspace; pred = M_f @ Wo; errors -
  for (int task = tid; task < fa * kD; task += kNT) {
    const int fl = task >> 4;
    attn_row_pass(sXA + fl * kD * kD, task & 15,
                  a.ws_as + ((size_t)s * F + f0 + fl) * kD * kD);
  }
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int task = tid; task < fa * Nmax; task += kNT) {
    const int fl = task / Nmax, n = task - fl * Nmax;
    float* pp = a.pred + ((size_t)s * F + f0 + fl) * kL2 * Nmax + n;
    if (n < nact) {
      float wo[kT];
#pragma unroll
      for (int t = 0; t < kT; ++t) wo[t] = sWo[t * Nmax + n];
      float y[kL2];
      const float* m = sM + fl * kL2 * kT;
#pragma unroll
      for (int jr = 0; jr < kL2; ++jr) {
        float x = 0.f;
#pragma unroll
        for (int t = 0; t < kT; ++t) x = fmaf(m[jr * kT + t], wo[t], x);
        y[jr] = x;
        pp[jr * Nmax] = x;        // pred_path_band = reshape(temp, (2, 12, N))
      }
      const bool has_t = a.ped_mask ? (a.ped_mask[(size_t)s * Nmax + n] != 0) : true;
      if (has_t) error_terms(y, sTgt + (fl * Nmax + n) * kL2, acc);
    } else {
#pragma unroll
      for (int jr = 0; jr < kL2; ++jr) pp[jr * Nmax] = 0.f;
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

template <int TPW>
__global__ void __launch_bounds__(kNT) g2k_recur_kernel(RecurArgs a) {
  __shared__ __attribute__((aligned(16))) float sAs[kRecurChunk * kD * kD];
  __shared__ __attribute__((aligned(16))) float sRed[2 * 128 + 128];
  __shared__ __attribute__((aligned(16))) float sT[4 * TPW * kTTile];
  const int s = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6, q = lane >> 4, j = lane & 15;
  const int F = a.F, H = a.H;
  const int nf = a.n_frames ? clampi(a.n_frames[s], 0, F) : F;
  STAMP(10);
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
  Recur<TPW> rec;
  rec.load(a.h_in + (size_t)s * kD * H, H, wv, q, j);
  if (nf > 0) {
    rec.init(sRed + 256, wv, q, j);
    for (int fb = 0; fb < nf; fb += kRecurChunk) {
      const int cnt = (nf - fb) < kRecurChunk ? (nf - fb) : kRecurChunk;
      dma_copy(a.att + ((size_t)s * F + fb) * kD * kD, sAs, cnt * (kD * kD / 4), wv, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (a.raw_attn) {
        for (int task = tid; task < cnt * kD; task += kNT)
          attn_column_pass(sAs + (task >> 4) * kD * kD, task & 15);
        __syncthreads();
        for (int task = tid; task < cnt * kD; task += kNT)
          attn_row_pass(sAs + (task >> 4) * kD * kD, task & 15, nullptr);
        __syncthreads();
      }
      STAMP(11);
      float4 arow = *reinterpret_cast<const float4*>(sAs + j * kD + 4 * q);
      for (int fl = 0; fl < cnt; ++fl)
        arow = rec.step(arow, fl + 1 < cnt ? sAs + (fl + 1) * kD * kD : nullptr,
                        sT + wv * TPW * kTTile, sRed + ((fb + fl) & 1) * 128, wv, q, j);
      __syncthreads();   // all waves done with sAs before the next DMA
    }
  }
  STAMP(12);
  rec.store(a.h_out + (size_t)s * kD * H, H, wv, q, j);
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
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
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

// Frames per g2k_frames_kernel workgroup: the largest chunk (<= 8) whose LDS
// carve stays within kFramesLdsBudget (>= 3 workgroups per CU), then
// balanced over the chunks.
struct StepPlan {
  int fchunk, nchunk;
  int64_t lds_bytes, ws_bytes;
};

StepPlan plan_step(const g2k_dims* d) {
  StepPlan p = {0, 0, 0, 0};
  const int F = d->F < 1 ? 1 : d->F;
  int best = 1;
  for (int fa = (F < 8 ? F : 8); fa >= 1; --fa) {
    if ((int64_t)frame_layout(d->Nmax, d->stride, fa).total * 4 <= kFramesLdsBudget) {
      best = fa;
      break;
    }
  }
  p.nchunk = (F + best - 1) / best;
  p.fchunk = (F + p.nchunk - 1) / p.nchunk;
  p.lds_bytes = (int64_t)frame_layout(d->Nmax, d->stride, p.fchunk).total * 4;
  const int64_t as_bytes = (int64_t)d->S * (d->F > 0 ? d->F : 0) * kD * kD * 4;
  p.ws_bytes = as_bytes + (int64_t)d->S * p.nchunk * 8 * 4;
  return p;
}

int launch_recur(const RecurArgs& r, int S, hipStream_t st) {
  switch (r.H / 64) {
    case 1: hipLaunchKernelGGL(g2k_recur_kernel<1>, dim3(S), dim3(kNT), 0, st, r); break;
    case 2: hipLaunchKernelGGL(g2k_recur_kernel<2>, dim3(S), dim3(kNT), 0, st, r); break;
    case 4: hipLaunchKernelGGL(g2k_recur_kernel<4>, dim3(S), dim3(kNT), 0, st, r); break;
    case 8: hipLaunchKernelGGL(g2k_recur_kernel<8>, dim3(S), dim3(kNT), 0, st, r); break;
    default: return set_err(G2K_EUNSUPPORTED, "H=%d: H/64 must be 1, 2, 4 or 8", r.H);
  }
  return G2K_OK;
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
  if (!workspace || workspace_bytes < p.ws_bytes)
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed (got %lld)", (long long)p.ws_bytes,
                   (long long)workspace_bytes);
  StepArgs a;
  a.d = *d; a.w = *w; a.pos = pos; a.vislet = vislet; a.G = G; a.targets = targets;
  a.n_active = n_active; a.n_frames = n_frames; a.ped_mask = ped_mask; a.h_in = h_in;
  a.h_out = h_out; a.pred = pred; a.metrics = metrics; a.A_out = A_out; a.cost_out = cost_out;
  a.lambda = lambda; a.fchunk = p.fchunk; a.nchunk = p.nchunk;
  a.ws_as = static_cast<float*>(workspace);
  a.ws_part = a.ws_as + (size_t)d->S * d->F * kD * kD;
  hipStream_t st = (hipStream_t)stream;
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

}  // extern "C"
