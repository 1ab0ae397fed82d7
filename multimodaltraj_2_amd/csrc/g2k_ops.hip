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
// one [16, 16] LDS tile whose first D rows / columns are real: column pass
// (running max, so exp never overflows: the ratio exp(a_r) / sum_{k<=r}
// exp(a_k) is shift-invariant) over rows < D, then row softmax over columns
// < D; padded rows and columns end as exact zeros.
__device__ __forceinline__ void attn_col(float* A, int c, int D) {
  float m = -INFINITY, s = 0.f;
  for (int r = 0; r < kD; ++r) {
    if (r >= D || c >= D) { A[r * kD + c] = 0.f; continue; }
    const float a = A[r * kD + c];
    const float mn = fmaxf(m, a);
    const float ea = __expf(a - mn);
    s = fmaf(s, __expf(m - mn), ea);
    m = mn;
    A[r * kD + c] = ea * rcp(s);
  }
}

__device__ __forceinline__ void attn_row(float* A, int r, int D) {
  float e[kD];
  float z = 0.f;
#pragma unroll
  for (int k = 0; k < kD; ++k) {
    e[k] = (r < D && k < D) ? __expf(A[r * kD + k]) : 0.f;
    z += e[k];
  }
  const float rz = r < D ? rcp(z) : 0.f;
#pragma unroll
  for (int k = 0; k < kD; ++k) A[r * kD + k] = e[k] * rz;
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
      for (int task = tid; task < cnt * kD; task += kRT) attn_col(sAs + (task >> 4) * kD * kD, task & 15, D);
      __syncthreads();
      for (int task = tid; task < cnt * kD; task += kRT) attn_row(sAs + (task >> 4) * kD * kD, task & 15, D);
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

__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + __expf(-x)); }

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
// GridLSTM cell on X[s][f][:D] with h[:, :2uK] as its state (16 lanes, one
// row each) into Xe, the one-feed forward (attn, cost, pred) from Xe, one
// recurrence frame on h — separated by workgroup barriers.  The same
// arithmetic as the three launches per frame (bit-identical), without a
// launch per body: the chain is latency-bound (one scene's worth of work per
// frame), so the launches were the cost.  (All global hand-offs stay inside
// the workgroup: its barriers order them; the CU's vector L1 is shared.)
// ---------------------------------------------------------------------------
struct ChainArgs {
  FwdArgs f;          // d (S = F = 1 per feed), weights, lambda
  GridArgs g;         // W, b, peep, state = h, state_out (scratch), rows = D, K
  const float *X, *Rel, *G;
  const int32_t *n_active, *n_frames;
  float *Xe, *attn, *cost, *pred, *h;
  int S, F, H;
};

template <int TPW, int U, int FS>
__global__ void __launch_bounds__(kNT) g2k_encoder_chain_kernel(ChainArgs a) {
  __shared__ FwdLds lf;
  __shared__ __attribute__((aligned(16))) float sAs[kD * kD];
  __shared__ __attribute__((aligned(16))) float sRed[4 * 16 * 4];
  const int Nmax = a.f.d.Nmax;
  const size_t xrow = (size_t)(kD + 2) * kD;
  for (int s = 0; s < a.S; ++s) {
    const int nf = clampi(a.n_frames[s], 0, a.F);
    for (int f = 0; f < nf; ++f) {
      const size_t sf = (size_t)s * a.F + f;
      if (threadIdx.x < kD) {                                     // train.py:201-207
        GridArgs g = a.g;
        g.in = a.X + sf * xrow;
        g.out = a.Xe + sf * xrow;
        gridlstm_row<U, FS>(g, threadIdx.x);
      }
      __syncthreads();
      FwdArgs w = a.f;                                            // g2k_lstm_mcr.py:99-124
      w.X = a.Xe + sf * xrow;
      w.Rel = a.Rel + (size_t)s * 2 * kD;
      w.G = a.G + (size_t)s * kD * kT;
      w.n_active = a.n_active + s;
      w.A_out = a.attn + sf * kD * kD;
      w.cost_out = a.cost + sf * kT * kT;
      w.pred = a.pred + sf * kL2 * Nmax;
      mcr_feed(w, 0, lf);
      __syncthreads();
      recur_scene<TPW, 4>(a.attn + sf * kD * kD, a.h, 0, 1, kD, a.H, sAs, sRed);   // :240-252
      __syncthreads();
    }
  }
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
