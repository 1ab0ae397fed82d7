// g2k_train.hip — train mode after the fused step (SURVEY.md §8(d) "--mode
// train", §8(e) gradient all-reduce): the per-scene gradient rows written
// by g2k_scene_kernel<..., GRAD> summed over scenes in a fixed order, and the
// optimizer update.  The reference has no loss or optimizer (SURVEY.md
// finding 5); the update follows the flags it parses (argParser.py:38-47).
#include "g2k_common.h"

namespace g2k {
namespace {

// grad[p] = sum_s rows[s][p]: workgroup = 32 columns x 32 row slices; slice
// k sums rows k, k + 32, ... in order with eight loads in flight (the rows
// one thread adds — 8 of the usual 256 — come in ONE memory round trip),
// then the 32 slices in order (the same sum for every launch: deterministic,
// no atomics on data).  UPD: the workgroup that finishes last then runs the
// optimizer step (opt_step) on the complete gradient.
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
  opt_step<true>(up.params, up.ms, grad, width - 2, up.lr, up.decay, up.clip, &red[0][0],
                 wave_id(), 16, threadIdx.x & 63, [] { __syncthreads(); });
}

__global__ void __launch_bounds__(1024) g2k_update_kernel(float* __restrict__ params,
                                                          float* __restrict__ ms,
                                                          const float* __restrict__ grad, int n,
                                                          float lr, float decay, float clip) {
  __shared__ float red[16];
  opt_step<false>(params, ms, grad, n, lr, decay, clip, red, wave_id(), 16, threadIdx.x & 63,
                  [] { __syncthreads(); });
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
