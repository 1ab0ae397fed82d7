// g2k_data.hip — device side of the tensorized data path (SURVEY.md §8(f)
// row 1): expands the walk plans of g2k_walk.cpp (CSV column per window slot
// and per target step) into the fused step's [S, ...] inputs, reading the
// split's positions and vislet rows resident in HBM.  Replaces the per-batch
// numpy of train.py:76-85 / sample.py:152-164 (node_pos_list -> window) and
// the target lists of networkx_graph.py:58-66, for S scenes in one launch.
#include "g2k_common.h"

namespace g2k {
namespace {

struct GatherArgs {
  const float* xy;        // [cols, 2]
  const float* vis;       // [2, cols] or NULL (ETH: no vislet rows, Q14)
  int64_t cols;
  const int32_t* pos_col; // [S, 8, Nmax]
  const int32_t* tgt_col; // [S, Nmax, 12]
  const int32_t* vis_off; // [S] or NULL (0)
  const int32_t* n_active;// [S]
  int S, F, Nmax;
  float* pos;             // [S, 8, Nmax, 2]
  float* vislet;          // [S, 2, Nmax]
  float* targets;         // [S, F, Nmax, 12, 2]
  uint8_t* ped_mask;      // [S, Nmax]
};

__device__ __forceinline__ float2 col_xy(const GatherArgs& a, int32_t c) {
  if (c < 0 || c >= a.cols) return make_float2(0.f, 0.f);
  return reinterpret_cast<const float2*>(a.xy)[c];
}

// One workgroup per scene: the window, the vislet slice, the ped mask, then
// the target rows written once per frame (coalesced float2 stores).
__global__ void __launch_bounds__(256) g2k_gather_kernel(GatherArgs a) {
  const int s = blockIdx.x, tid = threadIdx.x, Nmax = a.Nmax;
  const int nact = min(max(a.n_active[s], 0), Nmax);
  const int32_t* pc = a.pos_col + (size_t)s * 8 * Nmax;
  float2* pos = reinterpret_cast<float2*>(a.pos) + (size_t)s * 8 * Nmax;
  for (int i = tid; i < 8 * Nmax; i += 256) {
    const int n = i % Nmax;
    pos[i] = n < nact ? col_xy(a, pc[i]) : make_float2(0.f, 0.f);
  }
  const int off = a.vis_off ? a.vis_off[s] : 0;
  for (int i = tid; i < 2 * Nmax; i += 256) {
    const int r = i / Nmax, n = i % Nmax;
    const int64_t c = (int64_t)off + n;
    a.vislet[(size_t)s * 2 * Nmax + i] =
        (a.vis && n < nact && c >= 0 && c < a.cols) ? a.vis[r * a.cols + c] : 0.f;
  }
  const int32_t* tc = a.tgt_col + (size_t)s * Nmax * 12;
  for (int n = tid; n < Nmax; n += 256) {
    bool full = n < nact;
#pragma unroll
    for (int l = 0; l < 12; ++l) full = full && tc[n * 12 + l] >= 0 && tc[n * 12 + l] < a.cols;
    a.ped_mask[(size_t)s * Nmax + n] = full ? 1 : 0;
  }
  float2* tg = reinterpret_cast<float2*>(a.targets) + (size_t)s * a.F * Nmax * 12;
  const int per = Nmax * 12;
  for (int i = tid; i < per; i += 256) {
    const int n = i / 12;
    const float2 v = n < nact ? col_xy(a, tc[i]) : make_float2(0.f, 0.f);
    for (int f = 0; f < a.F; ++f) tg[(size_t)f * per + i] = v;
  }
}

}  // namespace
}  // namespace g2k

using namespace g2k;

extern "C" int g2k_scene_gather_f32(const float* xy, const float* vis, int64_t cols,
                                    const int32_t* pos_col, const int32_t* tgt_col,
                                    const int32_t* vis_off, const int32_t* n_active, int32_t S,
                                    int32_t F, int32_t Nmax, float* pos, float* vislet,
                                    float* targets, uint8_t* ped_mask, void* stream) {
  if (S < 0 || F < 1 || Nmax < 1 || Nmax > kMaxN || cols < 1)
    return set_err(G2K_EINVAL, "g2k_scene_gather_f32: S=%d F=%d Nmax=%d cols=%lld", S, F, Nmax,
                   (long long)cols);
  if (S == 0) return G2K_OK;
  if (!xy || !pos_col || !tgt_col || !n_active || !pos || !vislet || !targets || !ped_mask)
    return set_err(G2K_EINVAL, "g2k_scene_gather_f32: a required pointer is NULL");
  if (((uintptr_t)xy & 7u) || ((uintptr_t)pos & 7u) || ((uintptr_t)targets & 7u))
    return set_err(G2K_EINVAL, "g2k_scene_gather_f32: xy / pos / targets must be 8-byte aligned");
  GatherArgs a{xy, vis, cols, pos_col, tgt_col, vis_off, n_active, S, F, Nmax,
               pos, vislet, targets, ped_mask};
  hipLaunchKernelGGL(g2k_gather_kernel, dim3(S), dim3(256), 0, (hipStream_t)stream, a);
  return check_launch("g2k_scene_gather_f32");
}
