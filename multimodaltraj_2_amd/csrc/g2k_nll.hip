// g2k_nll.hip — the bivariate-Gaussian NLL head and its sampling path
// ("North-star NLL"; absent from the reference, so
// PARITY UNPINNED — oracle/g2k_ref.py restates it and pins the gradient by
// central finite differences).
//
// Head: per prediction step t a Gaussian around the model's prediction
// mu = pred_path_band[:, t, n] with sigma_x = exp(ls_x[t]), sigma_y =
// exp(ls_y[t]), rho = tanh(r[t]) (head [3][12] = ls_x, ls_y, r).  With
// a = (x - mu_x) / sigma_x, b = (y - mu_y) / sigma_y, c = 1 - rho^2,
// z = a^2 + b^2 - 2 rho a b:
//   nll = log(2 pi) + ls_x + ls_y + 1/2 log c + z / (2c)
//   d/dmu_x = -(a - rho b) / (c sigma_x)    d/dmu_y = -(b - rho a) / (c sigma_y)
//   d/dls_x = 1 - (a^2 - rho a b) / c       d/dls_y = 1 - (b^2 - rho a b) / c
//   d/dr    = -rho - a b + rho z / c
// summed over frames f < n_frames, active masked pedestrians and the 12 steps
// (the pairs the a9 errors and the L2 train loss use).
//
// g2k_nll_kernel: one workgroup per scene, 192 threads = 16 groups x 12
// steps (thread t-lane fixed, so its three head-gradient sums are registers);
// group g walks the scene's (frame, pedestrian) pairs g, g + 16, ...; the 16
// groups' sums are added in group order (deterministic) into the scene's row
// [38] = {d/dls_x[12], d/dls_y[12], d/dr[12], nll, pairs}; the rows are summed
// over scenes by g2k_grad_rows_kernel (fixed order).  dpred (optional) gets
// d nll / d pred in pred's layout (zero elsewhere in the active columns of
// frames < n_frames).
// g2k_gauss_sample_kernel: one thread per (s, f, t, n): x = mu_x + sigma_x e1,
// y = mu_y + sigma_y (rho e1 + sqrt(c) e2), (e1, e2) by Box-Muller from a
// counter-based hash of (seed, element) — reproducible, restated in the oracle.
#include "g2k_common.h"

namespace g2k {
namespace {

constexpr int kNllGroups = 16;
constexpr int kNllThreads = kNllGroups * kL;   // 192
constexpr int kNllRow = 3 * kL + 2;            // 38
constexpr float kLog2Pi = 1.8378770664093453f;

__global__ void __launch_bounds__(kNllThreads) g2k_nll_kernel(
    const float* __restrict__ pred, const float* __restrict__ targets,
    const int32_t* __restrict__ n_active, const int32_t* __restrict__ n_frames,
    const uint8_t* __restrict__ ped_mask, const float* __restrict__ head, int F, int Nmax,
    float* __restrict__ rows, float* __restrict__ dpred) {
  __shared__ float part[kNllGroups][kL][5];
  const int s = blockIdx.x;
  const int t = threadIdx.x % kL, g = threadIdx.x / kL;
  const int nact = clampi(n_active[s], 0, Nmax);
  const int nf = n_frames ? clampi(n_frames[s], 0, F) : F;
  const float lsx = head[t], lsy = head[kL + t], r = head[2 * kL + t];
  const float sx = expf(lsx), sy = expf(lsy), rho = tanhf(r);
  const float c = 1.f - rho * rho, ic = 1.f / c;
  const float isx = 1.f / sx, isy = 1.f / sy;
  const float base = kLog2Pi + lsx + lsy + 0.5f * logf(c);
  float gx = 0.f, gy = 0.f, gr = 0.f, nll = 0.f, pairs = 0.f;
  const int npair = nf * nact;
  for (int p = g; p < npair; p += kNllGroups) {
    const int f = p / nact, n = p - f * nact;
    const size_t pb = ((size_t)s * F + f) * kL2 * Nmax;
    const bool on = ped_mask ? ped_mask[(size_t)s * Nmax + n] != 0 : true;
    float dmx = 0.f, dmy = 0.f;
    if (on) {
      const float mx = pred[pb + (size_t)t * Nmax + n], my = pred[pb + (size_t)(kL + t) * Nmax + n];
      const float2 tg = reinterpret_cast<const float2*>(targets)[(((size_t)s * F + f) * Nmax + n) * kL + t];
      const float a = (tg.x - mx) * isx, b = (tg.y - my) * isy;
      const float z = a * a + b * b - 2.f * rho * a * b;
      nll += base + 0.5f * z * ic;
      dmx = -(a - rho * b) * ic * isx;
      dmy = -(b - rho * a) * ic * isy;
      gx += 1.f - (a * a - rho * a * b) * ic;
      gy += 1.f - (b * b - rho * a * b) * ic;
      gr += -rho - a * b + rho * z * ic;
      pairs += t == 0 ? 1.f : 0.f;
    }
    if (dpred) {
      dpred[pb + (size_t)t * Nmax + n] = dmx;
      dpred[pb + (size_t)(kL + t) * Nmax + n] = dmy;
    }
  }
  part[g][t][0] = gx; part[g][t][1] = gy; part[g][t][2] = gr;
  part[g][t][3] = nll; part[g][t][4] = pairs;
  __syncthreads();
  float* row = rows + (size_t)s * kNllRow;
  if (threadIdx.x < 3 * kL) {                   // head gradients: group order
    const int k = threadIdx.x / kL, tt = threadIdx.x % kL;
    float v = 0.f;
    for (int q = 0; q < kNllGroups; ++q) v += part[q][tt][k];
    row[threadIdx.x] = v;
  } else if (threadIdx.x < 3 * kL + 2) {        // nll, pairs: group order, then steps
    const int k = 3 + threadIdx.x - 3 * kL;
    float v = 0.f;
    for (int q = 0; q < kNllGroups; ++q)
      for (int tt = 0; tt < kL; ++tt) v += part[q][tt][k];
    row[threadIdx.x] = v;
  }
}

// 32-bit mix (PCG output permutation of an LCG step): the sampler's
// counter-based uniform source; restated in oracle/g2k_ref.py (gauss_sample)
__device__ __forceinline__ uint32_t pcg_hash(uint32_t v) {
  const uint32_t st = v * 747796405u + 2891336453u;
  const uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
  return (w >> 22u) ^ w;
}

__global__ void __launch_bounds__(256) g2k_gauss_sample_kernel(
    const float* __restrict__ pred, const float* __restrict__ head, int64_t total, int Nmax,
    uint32_t seed_lo, uint32_t seed_hi, float* __restrict__ out) {
  // element e = ((s * F + f) * 12 + t) * Nmax + n
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int n = (int)(e % Nmax);
  const int64_t sft = e / Nmax;
  const int t = (int)(sft % kL);
  const int64_t sf = sft / kL;
  const uint32_t key = pcg_hash(seed_lo ^ pcg_hash(seed_hi ^ (uint32_t)(e >> 32))) ^ (uint32_t)e;
  const uint32_t h1 = pcg_hash(2u * key + 1u), h2 = pcg_hash(2u * key + 2u);
  const float u1 = ((float)(h1 >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float u2 = ((float)(h2 >> 8) + 0.5f) * (1.0f / 16777216.0f);
  const float rad = sqrtf(-2.f * logf(u1));
  const float e1 = rad * cosf(6.283185307179586f * u2), e2 = rad * sinf(6.283185307179586f * u2);
  const float sx = expf(head[t]), sy = expf(head[kL + t]), rho = tanhf(head[2 * kL + t]);
  const size_t px = (size_t)(sf * kL2 + t) * Nmax + n, py = (size_t)(sf * kL2 + kL + t) * Nmax + n;
  out[px] = pred[px] + sx * e1;
  out[py] = pred[py] + sy * (rho * e1 + sqrtf(1.f - rho * rho) * e2);
}

}  // namespace

int nll_launch(const g2k_dims* d, const float* pred, const float* targets, const int32_t* n_active,
               const int32_t* n_frames, const uint8_t* ped_mask, const float* head, float* rows,
               float* dpred, hipStream_t st) {
  hipLaunchKernelGGL(g2k_nll_kernel, dim3(d->S), dim3(kNllThreads), 0, st, pred, targets, n_active,
                     n_frames, ped_mask, head, d->F, d->Nmax, rows, dpred);
  return check_launch("g2k_nll_kernel");
}

int gauss_sample_launch(const g2k_dims* d, const float* pred, const float* head, uint64_t seed,
                        float* out, hipStream_t st) {
  const int64_t total = (int64_t)d->S * d->F * kL * d->Nmax;
  hipLaunchKernelGGL(g2k_gauss_sample_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     pred, head, total, d->Nmax, (uint32_t)seed, (uint32_t)(seed >> 32), out);
  return check_launch("g2k_gauss_sample_kernel");
}

}  // namespace g2k
