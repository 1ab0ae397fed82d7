// recur1_probe — cycles per frame of the hidden-state recurrence (train.py:
// 240-252) held by ONE wave (all H = 128 columns: 8 tiles, no cross-wave
// exchange) against the scene kernel's four-wave form (chain_probe).  Per
// frame: row sums Z of e (in-lane over the tiles, then the 16 lanes of each
// row by DPP), A = split(As / Z), two split-f16 MFMAs per tile, exp2 and the
// next B split per tile, software-pipelined (tile t's exp under tile t+1's
// MFMAs).  One workgroup per CU; NX extra waves idle (0), poll LDS with
// s_sleep (1) or issue f32 MFMAs at priority 0 (2).  Development probe, not
// product code (timing only: the values are not checked).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I multimodaltraj_2_amd/csrc
//          -o tools/probes/recur1_probe tools/probes/recur1_probe.hip
#include <algorithm>
#include <cstdio>
#include <vector>
#include "g2k_recur.h"

using namespace g2k;

constexpr int kF = 64;

template <int EXTRA, int TILES>
__global__ void __launch_bounds__(1024) recur1(unsigned long long* out, float* hout) {
  __shared__ __attribute__((aligned(16))) float sAs[kF * 256];
  __shared__ int sDone;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, L = lane & 15, q = lane >> 4;
  for (int i = threadIdx.x; i < kF * 256; i += blockDim.x) {
    const int r = (i >> 4) & 15;
    sAs[i] = kLog2e / 16.f * (1.f + 0.01f * ((i * 7 + r) % 13));
  }
  if (threadIdx.x == 0) sDone = 0;
  __syncthreads();
  if (wv >= 1) {
    if (EXTRA == 0) return;
    if (EXTRA == 1) {
      poll_flag(&sDone, 1);
      return;
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float a = lane * 1e-3f, b = 1.f;
    for (int it = 0; it < 100000; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
      int d;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(d) : "v"(lds_addr(&sDone)) : "memory");
      if (__builtin_amdgcn_readfirstlane(d)) break;
    }
    hout[blockIdx.x * 1024 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
    return;
  }
  __builtin_amdgcn_s_setprio(2);
  u32x4v bo[TILES];
  float e[TILES][4];
#pragma unroll
  for (int t = 0; t < TILES; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) e[t][i] = 0.0078f * (1.f + 0.01f * (t + i + L));
    bo[t] = split4(e[t][0], e[t][1], e[t][2], e[t][3]);
  }
  float p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[i] = 0.f;
#pragma unroll
    for (int t = 0; t < TILES; ++t) p[i] += e[t][i];
  }
  float x[TILES][4];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int g = 0; g < kF; ++g) {
    const float4 b = *reinterpret_cast<const float4*>(sAs + g * 256 + L * 16 + 4 * q);
    // Z: the 16 lanes of each row (every lane of the row group gets it)
    float z[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) z[i] = row16_sum(p[i]);
    const u32x4v A = split4(b.x * rcp(z[0]), b.y * rcp(z[1]), b.z * rcp(z[2]), b.w * rcp(z[3]));
    const u32x4v A2 = {A[2], A[3], A[0], A[1]};
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[TILES];
#pragma unroll
    for (int t = 0; t < TILES; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, A), __builtin_bit_cast(f16x8, bo[t]),
                                                      f32x4{-kOff, -kOff, -kOff, -kOff}, 0, 0, 0);
#pragma unroll
    for (int t = 0; t < TILES; ++t)
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, A2), __builtin_bit_cast(f16x8, bo[t]),
                                                      acc[t], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = 0.f;
#pragma unroll
    for (int t = 0; t < TILES; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[t][i] = acc[t][i];
        e[t][i] = __builtin_amdgcn_exp2f(acc[t][i]);
        p[i] += e[t][i];
      }
      bo[t] = split4(e[t][0], e[t][1], e[t][2], e[t][3]);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) sDone = 1;
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < TILES; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) sum += x[t][i];
  hout[blockIdx.x * 1024 + threadIdx.x] = sum;
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int EXTRA, int TILES>
void run(const char* name, int waves) {
  const int nb = 256;
  unsigned long long* d;
  float* h;
  (void)hipMalloc(&d, nb * sizeof(unsigned long long));
  (void)hipMalloc(&h, (size_t)nb * 1024 * 4);
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((recur1<EXTRA, TILES>), dim3(nb), dim3(64 * waves), 0, 0, d, h);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> v(nb);
  (void)hipMemcpy(v.data(), d, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::sort(v.begin(), v.end());
  printf("one wave, %d tiles (H = %d), %-18s waves %2d: %.0f cycles per frame (median), max %.0f\n", TILES,
         16 * TILES, name, waves, (double)v[nb / 2] / kF, (double)v[nb - 1] / kF);
  (void)hipFree(d);
  (void)hipFree(h);
}

int main() {
  run<0, 8>("alone", 1);
  run<1, 8>("+15 polling waves", 16);
  run<2, 8>("+15 MFMA waves", 16);
  run<0, 4>("alone", 1);
  run<0, 16>("alone", 1);
  return 0;
}
