// g2k_ops.hip — the path's single-purpose operators behind the C ABI (besides
// the fused step in g2k_scene.hip):
//   g2k_recur_kernel        train.py:240-252 over F attention matrices
//                           (g2k_frame_recurrence_f32), D <= 16
//   g2k_mcr_forward_kernel  models/g2k_lstm_mcr.py:99-124 (class-level
//                           forward, g2k_mcr_forward_f32), D <= 16
//   g2k_errors_v0/v1_kernel train.py:636-674 / sample.py:21-82
//   g2k_sigmoid / g2k_row_softmax  nri_learned.py:16-28
//   g2k_gridlstm_kernel     helper.py GridLSTMCell encoders (a6)
//   g2k_encoder_chain_kernel --use_grid_lstm: cell -> forward -> recurrence
//                           per frame in one workgroup (g2k_encoder_chain_f32)
//   g2k_ctx_conv / reduce   train.py:92-113, 154-158 static context (a5)
// D < 16 (sample.py's num_freq_blocks = 10 and the reference checkpoints,
// SURVEY.md Appendix D) runs on the same 16-wide tiles with the rows and
// columns past D held at zero and masked out of every softmax.
#include "g2k_common.h"
#include "g2k_recur.h"

namespace g2k {
namespace {

constexpr int kRecurChunk = 32;   // As tiles resident in LDS

// As = softmax(exp(A) / cumsum(exp(A), axis=0), axis=-1) (train.py:240) of
// one [16, 16] LDS tile whose first D rows / columns are real, by ONE wave,
// in place: lane (L, q) holds column L, rows 4q .. 4q + 3.  Column pass: the
// ratio exp(A_r) / sum_{k<=r} exp(A_k) is shift-invariant, so with the
// column max M, e = exp(A - M) lies in (0, 1] and the prefix sums (in-lane,
// then across the lane groups by permlane swaps) cannot overflow; a column
// whose prefix sum underflows (its leading rows ~87 below its max) is redone
// with running (max, sum) pairs, exact for any finite A.  Then a 16-lane row
// softmax of values in (0, 1] (DPP).  Padded rows and columns end as exact
// zeros.  (The fused scene kernel's attn_weights in this kernel family's
// layout; a serial per-column walk of the 16 rows took ~2.2k cycles on the
// --use_grid_lstm chain, this ~0.5k.)
__device__ __forceinline__ void attn_tile_wave(float* A, int D, int lane) {
  const int L = lane & 15, q = lane >> 4;
  float aA[4];
  bool ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    aA[i] = A[(4 * q + i) * kD + L];
    ok[i] = L < D && 4 * q + i < D;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int i = 0; i < 4; ++i) mx = fmaxf(mx, ok[i] ? aA[i] : -INFINITY);
  mx = fmaxf(mx, partner16(mx));
  mx = fmaxf(mx, partner32(mx));
  float e[4], p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = ok[i] ? __expf(aA[i] - mx) : 0.f;
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
    bad |= ok[i] && !(P >= 1e-30f);
    R[i] = e[i] * rcp(P);
  }
  if (__builtin_amdgcn_ballot_w64(bad) != 0) {
    // running (max, sum exp) down the rows; exclusive prefix over the groups
    // (rows >= D only follow the real ones: they reach no real row's prefix)
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
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float ex = ok[i] ? __expf(R[i]) : 0.f;
    const float z = row16_sum(ex);
    A[(4 * q + i) * kD + L] = ok[i] ? ex * rcp(z) : 0.f;
  }
}

// ---------------------------------------------------------------------------
// Frame-sequential recurrence, one workgroup per scene, NW waves; the As of
// up to kRecurChunk frames staged in LDS, h in MFMA registers (g2k_recur.h).
// ---------------------------------------------------------------------------
// One scene's chain over F frames (sAs: min(F, kRecurChunk) As tiles; sRed:
// 4 * 16 * NW floats), the whole workgroup taking part
template <int TPW, int NW>
__device__ __forceinline__ void recur_scene(const float* __restrict__ att, float* __restrict__ h,
                                            int s, int F, int D, int H, float* sAs, float* sRed) {
  constexpr int kRT = 64 * NW;               // threads
  constexpr int kRB = 16 * NW;               // floats per row-partial buffer
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = wave_id(), q = lane >> 4, j = lane & 15;
  Recur<TPW, NW> rec;
  float* hs = h + (size_t)s * D * H;
  rec.load(hs, H, wv, q, j, D);
  const float* last = nullptr;
  if (F > 0) {
    rec.init_max(sRed + 3 * kRB, wv, q, j);
    __syncthreads();
    rec.init_exp(sRed, sRed + 3 * kRB, wv, q, j);   // published by the chunk barrier below
    int cur = 0;
    for (int fb = 0; fb < F; fb += kRecurChunk) {
      const int cnt = (F - fb) < kRecurChunk ? (F - fb) : kRecurChunk;
      const float* src = att + ((size_t)s * F + fb) * D * D;
      if (D == kD) {
        dma_copy_n<kRT>(src, sAs, cnt * (kD * kD / 4), wv, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        for (int i = tid; i < cnt * kD * kD; i += kRT) {
          const int f = i >> 8, r = (i >> 4) & 15, c = i & 15;
          sAs[i] = (r < D && c < D) ? src[(size_t)f * D * D + r * D + c] : 0.f;
        }
      }
      __syncthreads();
      for (int fl = wv; fl < cnt; fl += NW) attn_tile_wave(sAs + fl * kD * kD, D, lane);
      __syncthreads();
      for (int fl = 0; fl < cnt; ++fl) {
        const float4 b = *reinterpret_cast<const float4*>(sAs + fl * kD * kD + j * kD + 4 * q);
        const int nxt = cur == 2 ? 0 : cur + 1;
        rec.step(b, sRed + cur * kRB, sRed + nxt * kRB, wv, q, j);
        cur = nxt;
      }
      last = sRed + cur * kRB;
      __syncthreads();   // all waves done with sAs before the next chunk
    }
  }
  rec.store(hs, H, wv, q, j, last, D);
}

template <int TPW, int NW>
__global__ void __launch_bounds__(64 * NW) g2k_recur_kernel(const float* __restrict__ att,
                                                            float* __restrict__ h, int F, int D,
                                                            int H) {
  __shared__ __attribute__((aligned(16))) float sAs[kRecurChunk * kD * kD];
  __shared__ __attribute__((aligned(16))) float sRed[4 * 16 * NW];
  recur_scene<TPW, NW>(att, h, blockIdx.x, F, D, H, sAs, sRed);
}

// ---------------------------------------------------------------------------
// g2k_lstm_mcr.forward() only (models/g2k_lstm_mcr.py:99-124), one
// workgroup per feed, any D <= 16 (row-major [rows][D] operands):
//   g = lambda ngh; E = Wv @ X + bv; Rm = Wr @ Rel; A = g @ (E * Rm);
//   cost = E @ g; pred = reshape((Wc @ cost) @ Wo, (2, 12, N))
// ---------------------------------------------------------------------------
struct FwdArgs {
  g2k_dims d;
  g2k_weights w;
  const float *X, *Rel, *G;
  const int32_t* n_active;
  float *A_out, *cost_out, *pred;
  float lambda;
};

struct FwdLds {
  float X[(kD + 2) * kD], E[kT * kD], Rm[kT * kD], G[kD * kT], C[kT * kT], M[kL2 * kT];
};

// feed s of `a` by the whole (kNT-thread) workgroup
__device__ __forceinline__ void mcr_feed(const FwdArgs& a, int s, FwdLds& l) {
  float *sX = l.X, *sE = l.E, *sRm = l.Rm, *sG = l.G, *sC = l.C, *sM = l.M;
  const int tid = threadIdx.x;
  const int Nmax = a.d.Nmax, D = a.d.D;
  const int nact = clampi(a.n_active[s], 0, Nmax);
  for (int i = tid; i < (D + 2) * D; i += kNT) sX[i] = a.X[(size_t)s * (D + 2) * D + i];
  if (tid < D * kT) sG[tid] = a.lambda * a.G[(size_t)s * D * kT + tid];
  __syncthreads();
  if (tid < kT * D) {                           // E = Wv @ X + bv; Rm = Wr @ Rel
    const int t = tid / D, dc = tid - t * D;
    float e = 0.f;
    for (int k = 0; k < D + 2; ++k) e = fmaf(a.w.Wv[t * (D + 2) + k], sX[k * D + dc], e);
    sE[tid] = e + a.w.bv[dc];
    const float* rel = a.Rel + (size_t)s * 2 * D;
    sRm[tid] = fmaf(a.w.Wr[2 * t], rel[dc], a.w.Wr[2 * t + 1] * rel[D + dc]);
  }
  __syncthreads();
  if (tid < D * D) {                            // A = g @ (E * Rm)
    const int r = tid / D, dc = tid - r * D;
    float x = 0.f;
    for (int t = 0; t < kT; ++t) x = fmaf(sG[r * kT + t], sE[t * D + dc] * sRm[t * D + dc], x);
    a.A_out[(size_t)s * D * D + tid] = x;
  }
  if (tid < kT * kT) {                          // cost = E @ g
    const int t1 = tid >> 3, t2 = tid & 7;
    float c = 0.f;
    for (int k = 0; k < D; ++k) c = fmaf(sE[t1 * D + k], sG[k * kT + t2], c);
    sC[tid] = c;
    a.cost_out[(size_t)s * kT * kT + tid] = c;
  }
  __syncthreads();
  if (tid < kL2 * kT) {                         // M = Wc @ cost
    const int jr = tid >> 3, t2 = tid & 7;
    float x = 0.f;
    for (int t = 0; t < kT; ++t) x = fmaf(a.w.Wc[jr * kT + t], sC[t * kT + t2], x);
    sM[tid] = x;
  }
  __syncthreads();
  for (int i = tid; i < kL2 * Nmax; i += kNT) { // pred_path_band = M @ Wo
    const int jr = i / Nmax, n = i - jr * Nmax;
    float x = 0.f;
    if (n < nact)
      for (int t = 0; t < kT; ++t) x = fmaf(sM[jr * kT + t], a.w.Wo[t * Nmax + n], x);
    a.pred[(size_t)s * kL2 * Nmax + i] = x;
  }
}

__global__ void __launch_bounds__(kNT) g2k_mcr_forward_kernel(FwdArgs a) {
  __shared__ FwdLds l;
  mcr_feed(a, blockIdx.x, l);
}

// ---------------------------------------------------------------------------
// a2-a4 alone (train.py:76-85, 167-195), one workgroup per (scene, frame):
//   B = window norms [T, n] of rows f*stride + t; X0 = Wii @ (B @ Wi) [D, D];
//   Ve = vislet[:, :n] @ Wi [2, D]; X = [X0; Ve] (the outputs feed,
//   train.py:231); Rel = Ve * Ve (vislet_rel, train.py:194-195; frame 0's
//   workgroup writes it).  The model input of g2k_mcr_forward_f32, for the
//   per-frame chain of the --use_grid_lstm encoder stage (the GridLSTM's
//   output replaces X0 there).  D = 16.
// ---------------------------------------------------------------------------
struct EmbedArgs {
  g2k_dims d;
  g2k_weights w;
  const float *pos, *vislet;
  const int32_t* n_active;
  float *X, *Rel;
};

__global__ void __launch_bounds__(kNT) g2k_embed_kernel(EmbedArgs a) {
  __shared__ float sB[kT * kMaxN];
  __shared__ float sU[kT * kD];
  __shared__ float sVe[2 * kD];
  const int F = a.d.F, Nmax = a.d.Nmax;
  const int s = blockIdx.x / F, f = blockIdx.x - s * F, tid = threadIdx.x;
  const int n = clampi(a.n_active[s], 0, Nmax);
  for (int i = tid; i < kT * n; i += kNT) {        // a2: per-node L2 norm of the window rows
    const int t = i / n, p = i - t * n;
    const float2 xy = reinterpret_cast<const float2*>(a.pos)[((size_t)s * a.d.W + f * a.d.stride + t) * Nmax + p];
    sB[i] = sqrtf(fmaf(xy.x, xy.x, xy.y * xy.y));
  }
  __syncthreads();
  if (tid < kT * kD) {                              // U = B @ Wi
    const int t = tid >> 4, c = tid & 15;
    float u = 0.f;
    for (int p = 0; p < n; ++p) u = fmaf(sB[t * n + p], a.w.Wi[p * kD + c], u);
    sU[tid] = u;
  } else if (tid < kT * kD + 2 * kD) {              // a4: Ve = vislet @ Wi
    const int r = (tid - kT * kD) >> 4, c = tid & 15;
    const float* v = a.vislet + ((size_t)s * 2 + r) * Nmax;
    float e = 0.f;
    for (int p = 0; p < n; ++p) e = fmaf(v[p], a.w.Wi[p * kD + c], e);
    sVe[r * kD + c] = e;
  }
  __syncthreads();
  float* X = a.X + ((size_t)s * F + f) * (kD + 2) * kD;
  {                                                 // a3: X0 = Wii @ U (kNT == kD * kD)
    const int i = tid >> 4, c = tid & 15;
    float x = 0.f;
#pragma unroll
    for (int t = 0; t < kT; ++t) x = fmaf(a.w.Wii[i * kT + t], sU[t * kD + c], x);
    X[tid] = x;
  }
  if (tid < 2 * kD) {
    X[kD * kD + tid] = sVe[tid];
    if (f == 0 && a.Rel) a.Rel[(size_t)s * 2 * kD + tid] = sVe[tid] * sVe[tid];
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
  const int nact = clampi(a.n_active[s], 0, Nmax);
  const int nf = a.n_frames ? clampi(a.n_frames[s], 0, F) : F;
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
  const int nact = clampi(a.n_active[s], 0, Nmax);
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

// The cell's nonlinearities, branch-free and short (the --use_grid_lstm
// chain has two of them per frequency block on its critical path): sigmoid
// by v_exp + v_rcp (1 ulp); tanh as |x| + |x|^3 p(x^2) below 0.625 (the
// minimax odd polynomial the device library uses there) and 1 - 2 / (e^{2|x|}
// + 1) above, both formed and one selected (the library branches on |x| and
// a wave runs both paths).  |error| <= ~2e-7 against float64 (a6's
// restatement tolerance is 1e-4, tests/test_gridlstm.py).
__device__ __forceinline__ float sigmoid_f(float x) { return rcp(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float ax = fabsf(x), x2 = x * x;
  float p = fmaf(__int_as_float(0xbbbac73d), x2, __int_as_float(0x3ca908c9));
  p = fmaf(p, x2, __int_as_float(0xbd5c1c4e));
  p = fmaf(p, x2, __int_as_float(0x3e088382));
  p = fmaf(p, x2, __int_as_float(0xbeaaaa99));
  const float small = fmaf(x2, ax * p, ax);
  const float t = __builtin_amdgcn_exp2f(ax * (2.f * kLog2e));   // e^{2|x|} (inf: large = 1)
  const float large = fmaf(rcp(t + 1.f), -2.f, 1.f);
  return copysignf(ax < 0.625f ? small : large, x);
}

// One unit's gates from its three gate sums (coupled input / forget gates,
// peepholes p = (wIf, wIt, wOf, wOt), zero without them: the added terms
// are then exact zeros).  Written with explicit roundings (__fadd_rn /
// __fmul_rn are never contracted), so gridlstm_row and the chain's
// chain_cell produce the same bits whatever their surrounding code lets the
// compiler fuse.
struct CellGates {
  float cfn, ctn, mfn, mtn;
};
__device__ __forceinline__ CellGates cell_gates(float zi, float zj, float zo, float cf, float ct,
                                                const float (&p)[4]) {
  const float ig = sigmoid_f(__fadd_rn(zi, fmaf(p[0], cf, __fmul_rn(p[1], ct))));
  const float gg = tanh_f(zj);
  const float fg = __fsub_rn(1.f, ig), ing = __fmul_rn(ig, gg);
  const float cfn = fmaf(fg, cf, ing), ctn = fmaf(fg, ct, ing);
  const float og = sigmoid_f(__fadd_rn(zo, fmaf(p[2], cfn, __fmul_rn(p[3], ctn))));
  return CellGates{cfn, ctn, __fmul_rn(og, tanh_f(cfn)), __fmul_rn(og, tanh_f(ctn))};
}

template <int U, int FS>
__device__ __forceinline__ void gridlstm_row(const GridArgs& a, int64_t r) {
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
      float pj[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) pj[m] = peep ? a.peep[m * U + j] : 0.f;
      const CellGates gt = cell_gates(z[j], z[U + j], z[2 * U + j], cf[j], ct[j], pj);
      const float cfn = gt.cfn, ctn = gt.ctn, mfn = gt.mfn, mtn = gt.mtn;
      srow[2 * U * k + j] = ctn;
      srow[2 * U * k + U + j] = mtn;
      orow[2 * U * k + j] = mtn;
      orow[2 * U * k + U + j] = mfn;
      cf[j] = cfn;
      mf[j] = mfn;
    }
  }
}

template <int U, int FS>
__global__ void __launch_bounds__(256) g2k_gridlstm_kernel(GridArgs a) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= a.rows) return;
  gridlstm_row<U, FS>(a, r);
}

// ---------------------------------------------------------------------------
// --use_grid_lstm's encoder chain (train.py:197-252 with the encoder stage of
// :201-207; multimodaltraj_2_amd/encoder_step.py): ONE workgroup walks the
// frames of S batches in order, per frame the three bodies above — the
// GridLSTM cell on X[s][f][:D] with h[:, :2uK] as its state into Xe, the
// one-feed forward (attn, cost, pred) from Xe, one recurrence frame on h.
// The same arithmetic as the three launches per frame (bit-identical: every
// value is formed by the same operations in the same order), with every
// hand-off of the chain in LDS: h lives in LDS for the whole launch (read
// from / written to HBM once), the weights are staged once, a batch's G and
// Rm once per batch, the next frame's X is fetched into registers at the top
// of a frame and parked in LDS under its middle, and the outputs (Xe rows,
// the cell state, attn, cost, pred) are stores nothing waits for.  The cell
// runs one lane per (row, unit) — 16 U lanes, the units of a row exchanging
// their m_freq by lane permutes between frequency blocks — and a frame's
// pred (M @ Wo, which the chain never reads) is formed by waves 1..3 under
// the next frame's cell.  Per frame: six workgroup barriers (the row-max and
// numerator exchanges of the recurrence, the feed's three dependent stages,
// the h hand-off), no HBM round trip.
// ---------------------------------------------------------------------------
struct ChainArgs {
  FwdArgs f;          // d (Nmax), weights, lambda
  GridArgs g;         // W, b, peep, state_out (the cell state, written per frame)
  const float *X, *Rel, *G;
  const int32_t *n_active, *n_frames;
  float *Xe, *attn, *cost, *pred, *h;
  int S, F, H;
};

// m_freq of unit u of this lane's row: the row's U lanes are adjacent in one
// DPP quad (lane = r U + j), so a quad_perm broadcasts it — no LDS round trip
// between frequency blocks
template <int U, int u>
__device__ __forceinline__ float unit_bcast(float v) {
  if constexpr (U == 1) return v;
  else if constexpr (U == 2) return dpp<(u | u << 2 | (2 + u) << 4 | (2 + u) << 6)>(v);
  else return dpp<u * 0x55>(v);
}
template <int U, int u = 0>
__device__ __forceinline__ void units_bcast(float (&mf)[U], float v) {
  if constexpr (u < U) {
    mf[u] = unit_bcast<U, u>(v);
    units_bcast<U, u + 1>(mf, v);
  }
}

// One lane of the cell (row r, unit j): gridlstm_row's arithmetic for the
// unit's three gate columns.  cw[m][i] = W[i][m U + j], cb[m] = b[m U + j],
// cp[m] = peep[m U + j] (zero without peepholes, as gridlstm_row).  The dot
// products' terms over x_k and m_time (everything but m_freq, which comes
// last in their order) are formed for every block up front, so a block's
// critical path is U FMAs, the gates and the DPP broadcast.
template <int U, int FS>
__device__ __forceinline__ void chain_cell(const float (&cw)[3][FS + 2 * U], const float (&cb)[3],
                                           const float (&cp)[4], int r, int j, const float* xin,
                                           const float* hrow, float* xe, float* xe_g, float* st_g) {
  constexpr int NI = FS + 2 * U, K = kD / FS, NP = FS + U;
  float zp[K][3], ctk[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float v[NP];
#pragma unroll
    for (int i = 0; i < FS; ++i) v[i] = xin[r * kD + k * FS + i];          // x_k
#pragma unroll
    for (int u = 0; u < U; ++u) v[FS + u] = hrow[2 * U * k + U + u];        // m_time
    ctk[k] = hrow[2 * U * k + j];                                           // c_time
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float acc = cb[m];
#pragma unroll
      for (int i = 0; i < NP; ++i) acc = fmaf(v[i], cw[m][i], acc);
      zp[k][m] = acc;
    }
  }
  float cf = 0.f, mf[U];
#pragma unroll
  for (int u = 0; u < U; ++u) mf[u] = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float z[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      float acc = zp[k][m];
#pragma unroll
      for (int u = 0; u < U; ++u) acc = fmaf(mf[u], cw[m][NP + u], acc);  // m_freq of block k - 1
      z[m] = acc;
    }
    const CellGates gt = cell_gates(z[0], z[1], z[2], cf, ctk[k], cp);   // coupled: f = 1 - i
    const float cfn = gt.cfn, ctn = gt.ctn, mfn = gt.mfn, mtn = gt.mtn;
    st_g[r * kD + 2 * U * k + j] = ctn;
    st_g[r * kD + 2 * U * k + U + j] = mtn;
    xe[r * kD + 2 * U * k + j] = mtn;
    xe[r * kD + 2 * U * k + U + j] = mfn;
    xe_g[r * kD + 2 * U * k + j] = mtn;
    xe_g[r * kD + 2 * U * k + U + j] = mfn;
    cf = cfn;
    units_bcast<U>(mf, mfn);
  }
}

template <int TPW, int U, int FS>
__global__ void __launch_bounds__(kNT) g2k_encoder_chain_kernel(ChainArgs a) {
  constexpr int H = 64 * TPW;          // Recur<TPW, 4>: four waves of 16 TPW columns
  constexpr int HP = H + 4;            // h's LDS pitch: rows 4q + i of a lane group in distinct banks
  constexpr int NI = FS + 2 * U;
  constexpr int XR = (kD + 2) * kD;    // one frame's X / Xe
  __shared__ __attribute__((aligned(16))) float sH[kD * HP];
  __shared__ __attribute__((aligned(16))) float sXin[2][XR];
  __shared__ __attribute__((aligned(16))) float sXe[kD * kD];
  __shared__ __attribute__((aligned(16))) float sAs[kD * kD];
  __shared__ __attribute__((aligned(16))) float sRed[4 * 16 * 4];
  __shared__ float sWv[kT * (kD + 2)], sBv[kD], sWc[kL2 * kT], sWo[kT * kMaxN];
  __shared__ float sG[kD * kT], sRm[kT * kD], sE[kT * kD], sC[kT * kT], sM[kL2 * kT];
  const int tid = threadIdx.x, lane = tid & 63, wv = wave_id(), q = lane >> 4, L = lane & 15;
  const int Nmax = a.f.d.Nmax;
  const g2k_weights& w = a.f.w;
  for (int i = tid; i < kT * (kD + 2); i += kNT) sWv[i] = w.Wv[i];
  if (tid < kD) sBv[tid] = w.bv[tid];
  if (tid < kL2 * kT) sWc[tid] = w.Wc[tid];
  for (int i = tid; i < kT * Nmax; i += kNT) sWo[i] = w.Wo[i];
  for (int i = tid; i < kD * H; i += kNT) sH[(i / H) * HP + (i % H)] = a.h[i];
  const bool cell_lane = tid < kD * U;                 // wave 0
  const int cr = tid / U, cj = tid - (tid / U) * U;
  const bool peep = a.g.peep != nullptr;
  float cw[3][NI], cb[3], cp[4];   // cw: the x_k, m_time terms first, then m_freq (chain_cell)
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    cb[m] = cell_lane ? a.g.b[m * U + cj] : 0.f;
#pragma unroll
    for (int i = 0; i < NI; ++i) cw[m][i] = cell_lane ? a.g.W[i * 3 * U + m * U + cj] : 0.f;
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) cp[m] = (cell_lane && peep) ? a.g.peep[m * U + cj] : 0.f;

  // pred_path_band = M @ Wo of a finished frame (g2k_lstm_mcr.py:124)
  auto pred_of = [&](size_t psf, int pnact, int t0, int nt) {
    float* pp = a.pred + psf * kL2 * Nmax;
    for (int i = t0; i < kL2 * Nmax; i += nt) {
      const int jr = i / Nmax, n = i - jr * Nmax;
      float x = 0.f;
      if (n < pnact)
        for (int t = 0; t < kT; ++t) x = fmaf(sM[jr * kT + t], sWo[t * Nmax + n], x);
      pp[i] = x;
    }
  };
  int64_t pend_sf = -1;
  int pend_nact = 0;
#ifdef G2K_CHAIN_STAMPS   // development probe (tools/probes/chain_stamps.py): phase cycles into cost[.][32..41]
  uint64_t stamp[10];
#define CHAIN_STAMP(k) do { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); stamp[k] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define CHAIN_STAMP(k) do { } while (0)
#endif
  for (int s = 0; s < a.S; ++s) {
    const int nf = clampi(a.n_frames[s], 0, a.F);
    if (nf == 0) continue;
    const int nact = clampi(a.n_active[s], 0, Nmax);
    const size_t sf0 = (size_t)s * a.F;
    for (int i = tid; i < XR; i += kNT) sXin[0][i] = a.X[sf0 * XR + i];
    if (tid < kD * kT) sG[tid] = a.f.lambda * a.G[(size_t)s * kD * kT + tid];
    if (tid < kT * kD) {                               // Rm = Wr @ Rel (per batch)
      const int t = tid / kD, dc = tid - t * kD;
      const float* rel = a.Rel + (size_t)s * 2 * kD;
      sRm[tid] = fmaf(w.Wr[2 * t], rel[dc], w.Wr[2 * t + 1] * rel[kD + dc]);
    }
    __syncthreads();
    int cur = 0;
    for (int f = 0; f < nf; ++f) {
      const size_t sf = sf0 + f;
      const bool more = f + 1 < nf;
      CHAIN_STAMP(0);
      float px0 = 0.f, px1 = 0.f;                      // the next frame's X, parked in step 4
      if (more) {
        px0 = a.X[(sf + 1) * XR + tid];
        if (tid < XR - kNT) px1 = a.X[(sf + 1) * XR + kNT + tid];
      }
      // 1. h rows' maxima; the cell (train.py:201-207) | the previous frame's pred
      Recur<TPW, 4> rec;
      rec.load(sH, HP, wv, q, L);
      rec.init_max(sRed + 192, wv, q, L);
      CHAIN_STAMP(1);
      if (wv == 0) {
        if (cell_lane)
          chain_cell<U, FS>(cw, cb, cp, cr, cj, sXin[cur], sH + cr * HP, sXe, a.Xe + sf * XR,
                            a.g.state_out);
      } else if (pend_sf >= 0) {
        pred_of((size_t)pend_sf, pend_nact, tid - 64, kNT - 64);
      }
      CHAIN_STAMP(2);
      __syncthreads();
      CHAIN_STAMP(3);
      // 2. E = Wv @ X + bv (g2k_lstm_mcr.py:99-124); softmax numerators of h
      if (tid < kT * kD) {
        const int t = tid / kD, dc = tid - t * kD;
        float e = 0.f;
#pragma unroll
        for (int k = 0; k < kD + 2; ++k)
          e = fmaf(sWv[t * (kD + 2) + k], k < kD ? sXe[k * kD + dc] : sXin[cur][k * kD + dc], e);
        sE[tid] = e + sBv[dc];
      }
      rec.init_exp(sRed, sRed + 192, wv, q, L);
      __syncthreads();
      CHAIN_STAMP(4);
      // 3. A = g @ (E * Rm), cost = E @ g
      {
        const int r = tid / kD, dc = tid - r * kD;
        float x = 0.f;
        for (int t = 0; t < kT; ++t) x = fmaf(sG[r * kT + t], sE[t * kD + dc] * sRm[t * kD + dc], x);
        a.attn[sf * kD * kD + tid] = x;
        sAs[tid] = x;
      }
      if (tid < kT * kT) {
        const int t1 = tid >> 3, t2 = tid & 7;
        float c = 0.f;
        for (int k = 0; k < kD; ++k) c = fmaf(sE[t1 * kD + k], sG[k * kT + t2], c);
        sC[tid] = c;
        a.cost[sf * kT * kT + tid] = c;
      }
      __syncthreads();
      CHAIN_STAMP(5);
      // 4. As (train.py:240) on wave 0 | M = Wc @ cost on waves 1..3; next X parked
      if (more) {
        sXin[cur ^ 1][tid] = px0;
        if (tid < XR - kNT) sXin[cur ^ 1][kNT + tid] = px1;
      }
      if (wv == 0) {
        attn_tile_wave(sAs, kD, lane);
        CHAIN_STAMP(6);
      } else {
        const int i = tid - 64, jr = i >> 3, t2 = i & 7;
        float x = 0.f;
        for (int t = 0; t < kT; ++t) x = fmaf(sWc[jr * kT + t], sC[t * kT + t2], x);
        sM[i] = x;
      }
      __syncthreads();
      CHAIN_STAMP(7);
      // 5. the recurrence frame (train.py:243-252; its barrier inside), h back to LDS
      const float4 b = *reinterpret_cast<const float4*>(sAs + L * kD + 4 * q);
      rec.step(b, sRed, sRed + 64, wv, q, L);
      CHAIN_STAMP(8);
      rec.store(sH, HP, wv, q, L, sRed + 64);
      pend_sf = (int64_t)sf;
      pend_nact = nact;
      cur ^= 1;
      __syncthreads();
      CHAIN_STAMP(9);
#ifdef G2K_CHAIN_STAMPS
      if (tid == 0)
        for (int k = 1; k < 10; ++k) a.cost[sf * kT * kT + 32 + k] = (float)(stamp[k] - stamp[k - 1]);
#endif
    }
  }
  if (pend_sf >= 0) pred_of((size_t)pend_sf, pend_nact, tid, kNT);
  for (int i = tid; i < kD * H; i += kNT) a.h[i] = sH[(i / H) * HP + (i % H)];
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

}  // namespace

// Waves per recurrence workgroup: 4 (one per SIMD); 8 measured 0-5 % slower.
int recur_launch(const float* A, float* h, int S, int frames, int D, int H, hipStream_t st) {
  const dim3 g(S), b(256);
  switch (H / 64) {
    case 1: hipLaunchKernelGGL((g2k_recur_kernel<1, 4>), g, b, 0, st, A, h, frames, D, H); break;
    case 2: hipLaunchKernelGGL((g2k_recur_kernel<2, 4>), g, b, 0, st, A, h, frames, D, H); break;
    case 4: hipLaunchKernelGGL((g2k_recur_kernel<4, 4>), g, b, 0, st, A, h, frames, D, H); break;
    case 8: hipLaunchKernelGGL((g2k_recur_kernel<8, 4>), g, b, 0, st, A, h, frames, D, H); break;
    default: return set_err(G2K_EUNSUPPORTED, "H=%d unsupported", H);
  }
  return check_launch("g2k_frame_recurrence_f32");
}

int mcr_forward_launch(const g2k_dims* d, const g2k_weights* w, const float* X, const float* Rel,
                       const float* G, const int32_t* n_active, float* A_out, float* cost_out,
                       float* pred, float lambda, hipStream_t st) {
  FwdArgs a;
  a.d = *d; a.w = *w; a.X = X; a.Rel = Rel; a.G = G; a.n_active = n_active; a.A_out = A_out;
  a.cost_out = cost_out; a.pred = pred; a.lambda = lambda;
  hipLaunchKernelGGL(g2k_mcr_forward_kernel, dim3(d->S), dim3(kNT), 0, st, a);
  return check_launch("g2k_mcr_forward_f32");
}

int embed_launch(const g2k_dims* d, const g2k_weights* w, const float* pos, const float* vislet,
                 const int32_t* n_active, float* X, float* Rel, hipStream_t st) {
  static_assert(kNT == kD * kD, "one thread per X0 entry");
  EmbedArgs a;
  a.d = *d; a.w = *w; a.pos = pos; a.vislet = vislet; a.n_active = n_active; a.X = X; a.Rel = Rel;
  hipLaunchKernelGGL(g2k_embed_kernel, dim3((unsigned)((int64_t)d->S * d->F)), dim3(kNT), 0, st, a);
  return check_launch("g2k_frame_embed_f32");
}

int errors_launch(const g2k_dims* d, const float* pred, const float* targets,
                  const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                  int variant, float* out, hipStream_t st) {
  ErrArgs a;
  a.d = *d; a.pred = pred; a.targets = targets; a.n_active = n_active; a.n_frames = n_frames;
  a.ped_mask = ped_mask; a.out = out;
  if (variant == 0)
    hipLaunchKernelGGL(g2k_errors_v0_kernel, dim3(d->S), dim3(kNT), 0, st, a);
  else
    hipLaunchKernelGGL(g2k_errors_v1_kernel, dim3(d->S), dim3(64), 0, st, a);
  return check_launch("g2k_ade_fde_f32");
}

int relation_launch(const float* adj, float* out, int64_t rows, int cols, bool softmax,
                    hipStream_t st) {
  if (softmax) {
    hipLaunchKernelGGL(g2k_row_softmax_kernel, dim3((unsigned)rows), dim3(64), 0, st, adj, out, cols);
    return check_launch("g2k_eval_rln_ngh_f32");
  }
  const int64_t n = rows * (int64_t)cols;
  hipLaunchKernelGGL(g2k_sigmoid_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, adj,
                     out, n);
  return check_launch("g2k_infer_rlns_f32");
}

int encoder_chain_launch(const g2k_dims* d, const g2k_weights* w, const float* X, const float* Rel,
                         const float* G, const int32_t* n_active, const int32_t* n_frames,
                         const float* cell_W, const float* cell_b, const float* cell_peep,
                         int feature_size, int num_units, float* Xe, float* cell_state, float* attn,
                         float* cost, float* pred, float* h, float lambda, hipStream_t st) {
  ChainArgs a;
  a.f.d = *d;
  a.f.d.S = 1; a.f.d.F = 1; a.f.d.H = 64; a.f.d.W = kT; a.f.d.stride = 0; a.f.d.flags = 0;
  a.f.w = *w; a.f.lambda = lambda;
  a.g.state = h; a.g.ld_state = d->H; a.g.W = cell_W; a.g.b = cell_b; a.g.peep = cell_peep;
  a.g.state_out = cell_state; a.g.rows = kD; a.g.ld_in = kD; a.g.K = kD / feature_size;
  a.X = X; a.Rel = Rel; a.G = G; a.n_active = n_active; a.n_frames = n_frames;
  a.Xe = Xe; a.attn = attn; a.cost = cost; a.pred = pred; a.h = h;
  a.S = d->S; a.F = d->F; a.H = d->H;
#define G2K_CHAIN(T)                                                                            \
  switch (num_units) {                                                                          \
    case 1: hipLaunchKernelGGL((g2k_encoder_chain_kernel<T, 1, 2>), dim3(1), dim3(kNT), 0, st, a); break; \
    case 2: hipLaunchKernelGGL((g2k_encoder_chain_kernel<T, 2, 4>), dim3(1), dim3(kNT), 0, st, a); break; \
    default: hipLaunchKernelGGL((g2k_encoder_chain_kernel<T, 4, 8>), dim3(1), dim3(kNT), 0, st, a); break; \
  }
  switch (d->H / 64) {
    case 1: G2K_CHAIN(1) break;
    case 2: G2K_CHAIN(2) break;
    case 4: G2K_CHAIN(4) break;
    case 8: G2K_CHAIN(8) break;
    default: return set_err(G2K_EUNSUPPORTED, "H=%d unsupported", d->H);
  }
#undef G2K_CHAIN
  return check_launch("g2k_encoder_chain_f32");
}

int gridlstm_launch(const float* in, int64_t ld_in, const float* state, int64_t ld_state,
                    const float* W, const float* b, const float* peep, float* out, float* state_out,
                    int64_t rows, int blocks, int feature_size, int num_units, hipStream_t st) {
  GridArgs a;
  a.in = in; a.state = state; a.W = W; a.b = b; a.peep = peep; a.out = out; a.state_out = state_out;
  a.rows = rows; a.ld_in = ld_in; a.ld_state = ld_state; a.K = blocks;
  const dim3 g((unsigned)((rows + 255) / 256)), blk(256);
  switch (num_units * 16 + feature_size) {
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

int ctx_conv_launch(const float* img, int Hh, int Ww, int C, const float* filt, int D, float lambda,
                    float* out, float* G, float* part, hipStream_t st) {
  CtxArgs a;
  a.img = img; a.filt = filt; a.part = part; a.out = out; a.G = G;
  a.Hh = Hh; a.Ww = Ww; a.C = C; a.D = D; a.KH = Hh + 3 - D; a.KW = Ww + 2 - D; a.lambda = lambda;
  const size_t lds = (size_t)4 * (((a.KW * C + 3) & ~3) + (size_t)D * (Ww + 1) * C);
  if (lds > 160 * 1024) return set_err(G2K_ELDS, "image width %d needs %zu bytes of LDS", Ww, lds);
  hipLaunchKernelGGL(g2k_ctx_conv_kernel, dim3(a.KH), dim3(256), lds, st, a);
  hipLaunchKernelGGL(g2k_ctx_reduce_kernel, dim3(D), dim3(256), 0, st, a);
  return check_launch("g2k_context_conv_f32");
}

}  // namespace g2k
