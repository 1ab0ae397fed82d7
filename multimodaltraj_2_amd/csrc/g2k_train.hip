// g2k_train.hip — train mode after the fused step (SURVEY.md §8(d) "--mode
// train", §8(e) gradient all-reduce): the per-scene gradient rows written
// by g2k_scene_kernel<..., GRAD> summed over scenes in a fixed order, and the
// optimizer update.  The reference has no loss or optimizer (SURVEY.md
// finding 5); the update follows the flags it parses (argParser.py:38-47).
#include "g2k_common.h"

namespace g2k {
namespace {

// Optimizer step (argParser.py:38-47: grad_clip, learning_rate, decay_rate):
// g = grad / count, clipped by global norm (g * clip / max(||g||, clip)),
// then RMSProp (ms = decay ms + (1 - decay) g^2; p -= lr g / sqrt(ms +
// 1e-10), TF RMSPropOptimizer without momentum) or SGD (ms NULL).  One
// workgroup of 1024: the norm is a fixed-order block reduction.  COH: the
// gradient is read with agent-scope atomic loads (it was just written by
// other workgroups of the same launch, see g2k_grad_rows_kernel).
template <bool COH>
__device__ __forceinline__ float grad_at(const float* g, int i) {
  if (COH) return __hip_atomic_load(const_cast<float*>(g + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return g[i];
}

constexpr int kPre = 8;   // entries per thread held in registers (n <= 8192)

// this thread's parameters and mean squares (entries tid + 1024 j), loaded
// ahead of the gradient they are updated with
__device__ __forceinline__ void load_update_state(const float* __restrict__ params,
                                                  const float* __restrict__ ms, int n,
                                                  float (&pp)[kPre], float (&pm)[kPre]) {
#pragma unroll
  for (int j = 0; j < kPre; ++j) {
    const int i = threadIdx.x + j * 1024;
    pp[j] = i < n ? params[i] : 0.f;
    pm[j] = (ms && i < n) ? ms[i] : 0.f;
  }
}

// PRE: pp / pm already hold this thread's parameters and mean squares
// (load_update_state; n <= kPre * 1024)
template <bool COH, bool PRE = false>
__device__ __forceinline__ void update_body(float* __restrict__ params, float* __restrict__ ms,
                                            const float* __restrict__ grad, int n, float lr,
                                            float decay, float clip, float* red,
                                            float (*ppre)[kPre] = nullptr,
                                            float (*pmre)[kPre] = nullptr) {
  const int tid = threadIdx.x;
  // up to kPre entries per thread: parameters and mean squares are loaded
  // together with the gradient, before the norm's reduction
  const bool pre = n <= kPre * 1024;
  float pg[kPre], pp[kPre], pm[kPre];
  if (pre) {
    if (PRE) {
#pragma unroll
      for (int j = 0; j < kPre; ++j) { pp[j] = (*ppre)[j]; pm[j] = (*pmre)[j]; }
    } else {
      load_update_state(params, ms, n, pp, pm);
    }
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const int i = tid + j * 1024;
      pg[j] = i < n ? grad_at<COH>(grad, i) : 0.f;
    }
  }
  const float inv = 1.0f / fmaxf(grad_at<COH>(grad, n + 1), 1.0f);
  float ss = 0.f;
  if (pre) {
#pragma unroll
    for (int j = 0; j < kPre; ++j) {
      const float g = pg[j] * inv;
      ss = fmaf(g, g, ss);
    }
  } else {
    for (int i = tid; i < n; i += 1024) {
      const float g = grad_at<COH>(grad, i) * inv;
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
    const float g = grad_at<COH>(grad, i) * scale;
    if (ms) {
      const float m = fmaf(decay, ms[i], (1.f - decay) * g * g);
      ms[i] = m;
      params[i] -= lr * g / sqrtf(m + 1e-10f);
    } else {
      params[i] = fmaf(-lr, g, params[i]);
    }
  }
}

// grad[p] = sum_s rows[s][p]: workgroup = 32 columns x 32 row slices; slice
// k sums rows k, k + 32, ... in order with eight loads in flight (the rows
// one thread adds — 8 of the usual 256 — come in ONE memory round trip),
// then the 32 slices in order (the same sum for every launch: deterministic,
// no atomics on data).  UPD: the workgroup that finishes last then runs the
// optimizer step on the complete gradient (one launch fewer per train step).
// The hand-off uses agent-scope atomics only — gradient stores that write
// through to the coherence point (sc1), their completion (vmcnt(0)) before
// the ticket's fetch-add, coherent loads by the last workgroup — so no L2
// write-back / invalidate is needed (a __threadfence() here costs a full L2
// write-back and invalidate per workgroup: measured +8 us per step).
constexpr int kRowSlices = 32, kRowCols = 32;
template <bool UPD>
__global__ void __launch_bounds__(kRowCols * kRowSlices) g2k_grad_rows_kernel(const float* __restrict__ rows,
                                                                              int S, int width,
                                                                              float* __restrict__ grad,
                                                                              UpdateArgs up) {
  __shared__ float red[kRowSlices][kRowCols + 1];
  __shared__ int last;
  const int c = threadIdx.x % kRowCols, sl = threadIdx.x / kRowCols;
  const int p = blockIdx.x * kRowCols + c;
  // UPD: the update's parameters and mean squares in flight with the rows
  // (only the last workgroup uses them: one memory round trip off its tail)
  float pp[kPre], pm[kPre];
  const bool pre = UPD && width - 2 <= kPre * 1024;
  if (pre) load_update_state(up.params, up.ms, width - 2, pp, pm);
  float acc = 0.f;
  if (p < width) {
    for (int r0 = sl; r0 < S; r0 += 8 * kRowSlices) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = r0 + i * kRowSlices;
        v[i] = rows[(size_t)(r < S ? r : S - 1) * width + p];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += r0 + i * kRowSlices < S ? v[i] : 0.f;
    }
  }
  red[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && p < width) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kRowSlices; ++k) t += red[k][c];
    if (UPD) __hip_atomic_store(grad + p, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else grad[p] = t;
  }
  if (!UPD) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this thread's column stored
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(up.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (int)gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  // the acquire side of the hand-off, in the last workgroup only (once per
  // step): the other workgroups' gradient columns happen-before its loads
  // under the HIP memory model, not just by gfx950's store ordering (their
  // write-through stores completed, vmcnt(0), before their ticket increments)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (pre)
    update_body<true, true>(up.params, up.ms, grad, width - 2, up.lr, up.decay, up.clip, &red[0][0],
                            &pp, &pm);
  else
    update_body<true>(up.params, up.ms, grad, width - 2, up.lr, up.decay, up.clip, &red[0][0]);
}

__global__ void __launch_bounds__(1024) g2k_update_kernel(float* __restrict__ params,
                                                          float* __restrict__ ms,
                                                          const float* __restrict__ grad, int n,
                                                          float lr, float decay, float clip) {
  __shared__ float red[16];
  update_body<false>(params, ms, grad, n, lr, decay, clip, red);
}

}  // namespace

int grad_rows_launch(const float* rows, int S, int width, float* grad, hipStream_t st,
                     const UpdateArgs* up) {
  const dim3 grid((width + kRowCols - 1) / kRowCols), block(kRowCols * kRowSlices);
  if (up) {
    hipLaunchKernelGGL(g2k_grad_rows_kernel<true>, grid, block, 0, st, rows, S, width, grad, *up);
  } else {
    hipLaunchKernelGGL(g2k_grad_rows_kernel<false>, grid, block, 0, st, rows, S, width, grad,
                       UpdateArgs{});
  }
  return check_launch("g2k_grad_rows_kernel");
}

int update_launch(float* params, float* ms, const float* grad, int n, float lr, float decay,
                  float clip, hipStream_t st) {
  hipLaunchKernelGGL(g2k_update_kernel, dim3(1), dim3(1024), 0, st, params, ms, grad, n, lr, decay,
                     clip);
  return check_launch("g2k_update_kernel");
}

}  // namespace g2k
