// chain_probe — cycles per frame of the scene kernel's recurrence chain
// (Recur / RecurH step_seq, poll_red exchange) in isolation: one workgroup
// per CU, 4 recurrence waves (one per SIMD) running F frames over As tiles
// already in LDS, plus NX extra waves that either leave at once (idle), poll
// an LDS word with s_sleep (as waiting producers do), or issue f32 MFMAs at
// priority 0 (busy producers).  Development probe, not product code.
// build: hipcc --offload-arch=gfx950 -O3 -I include -I multimodaltraj_2_amd/csrc
//          -o tools/probes/chain_probe tools/probes/chain_probe.hip
#include <algorithm>
#include <cstdio>
#include <vector>
#include "g2k_recur.h"

using namespace g2k;

constexpr int kF = 64;
constexpr int kRB = 128;

template <bool H16, int EXTRA, int NW = 4>   // EXTRA: 0 idle, 1 poll+sleep, 2 MFMA spam
__global__ void __launch_bounds__(1024) chain(unsigned long long* out, float* hout) {
  __shared__ __attribute__((aligned(16))) float sAs[kF * 256];
  __shared__ __attribute__((aligned(16))) float sRed[4 * kRB];
  constexpr int TPW = 8 / NW;
  __shared__ int sFlag[kF];
  __shared__ int sDone;
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, L = lane & 15, q = lane >> 4;
  for (int i = threadIdx.x; i < kF * 256; i += blockDim.x) {
    const int r = (i >> 4) & 15;
    sAs[i] = kLog2e / 16.f * (1.f + 0.01f * ((i * 7 + r) % 13));   // rows ~ 1/16 (not normalised: timing only)
  }
  for (int i = threadIdx.x; i < kF; i += blockDim.x) sFlag[i] = i + 1;
  if (threadIdx.x == 0) sDone = 0;
  int* seq = reinterpret_cast<int*>(sRed + 2 * kRB);
  if (threadIdx.x < NW) seq[threadIdx.x] = 0;
  __syncthreads();
  if (wv >= NW) {
    if (EXTRA == 0) return;
    if (EXTRA == 1) {
      poll_flag(&sDone, 1);
      return;
    }
    // MFMA spam until the chain is done
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    float a = lane * 1e-3f, b = 1.f;
    for (int it = 0; it < 100000; ++it) {
#pragma unroll
      for (int k = 0; k < 8; ++k) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
      int d;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(d) : "v"(lds_addr(&sDone)) : "memory");
      if (__builtin_amdgcn_readfirstlane(d)) break;
    }
    if (acc[0] == 12345.f) hout[0] = acc[1];
    return;
  }
  __builtin_amdgcn_s_setprio(2);
  float* hs = hout + (size_t)blockIdx.x * 16 * 128;
  for (int i = lane; i < 16 * 16 * TPW; i += 64) hs[(i / (16 * TPW)) * 128 + wv * 16 * TPW + (i % (16 * TPW))] = 0.01f * (i & 7);
  __builtin_amdgcn_s_waitcnt(0);
  typename std::conditional<H16, RecurH<TPW, NW>, Recur<TPW, NW>>::type rc;
  rc.load(hs, 128, wv, q, L);
  rc.init_max(sRed + 3 * kRB, wv, q, L);
  if (lane == 0) lds_store_flag(seq + wv, 1);
  poll_seq(seq + (L & (NW - 1)), 1);
  rc.init_exp(sRed, sRed + 3 * kRB, wv, q, L);
  asm volatile("" ::: "memory");
  if (lane == 0) lds_store_flag(seq + wv, 2);
  const float* as_lane = sAs + L * 16 + 4 * q;
  float4 b0, b1;
  int f0 = read_as(sFlag, as_lane, b0), f1 = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  auto frame = [&](int g, float4& b, int& flq, float4& bn, int& fln) {
    f32x4 zq;
    poll_red(seq + (L & (NW - 1)), g + 2, sRed + (g & 1) * kRB + (L & (NW - 1)) * 16 + 4 * q, zq);
    if (__builtin_amdgcn_readfirstlane(flq) != g + 1) wait_as(sFlag + g, g + 1, as_lane + g * 256, b);
    const int fn = g + 1 < kF ? g + 1 : g;
    if constexpr (H16) {
      rc.step_seq(b, zq, sRed + ((g + 1) & 1) * kRB, seq, g + 3, wv, q, L, sFlag + fn, as_lane + fn * 256,
                  fln, bn, g + 1 == kF);
    } else {
      rc.step_seq(b, zq, sRed + ((g + 1) & 1) * kRB, seq, g + 3, wv, q, L, sFlag + fn, as_lane + fn * 256,
                  fln, bn);
    }
  };
  for (int g = 0; g < kF; g += 2) {
    frame(g, b0, f0, b1, f1);
    frame(g + 1, b1, f1, b0, f0);
  }
  for (int w = 0; w < NW; w += 4) poll_seq_all(seq + w, kF + 2);
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_setprio(0);
  if (lane == 0 && wv == 0) lds_store_flag(&sDone, 1);
  rc.store(hs, 128, wv, q, L, sRed + (kF & 1) * kRB);
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <bool H16, int EXTRA, int NW = 4>
void run(int nwaves, const char* name) {
  const int nb = 256;
  unsigned long long* d;
  float* h;
  hipMalloc(&d, nb * sizeof(unsigned long long));
  hipMalloc(&h, (size_t)nb * 16 * 128 * 4);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((chain<H16, EXTRA, NW>), dim3(nb), dim3(64 * nwaves), 0, 0, d, h);
  hipDeviceSynchronize();
  std::vector<unsigned long long> v(nb);
  hipMemcpy(v.data(), d, nb * 8, hipMemcpyDeviceToHost);
  std::sort(v.begin(), v.end());
  printf("%-8s NW %d %-22s waves %2d: %.0f cycles per frame (median over 256 WGs), max %.0f\n", H16 ? "h16" : "f32", NW, name,
         nwaves, (double)v[nb / 2] / kF, (double)v.back() / kF);
  hipFree(d);
  hipFree(h);
}

int main() {
  run<false, 0>(4, "alone");
  run<true, 0>(4, "alone");
  run<false, 1>(16, "+12 polling waves");
  run<true, 1>(16, "+12 polling waves");
  run<false, 2>(16, "+12 MFMA waves");
  run<true, 2>(16, "+12 MFMA waves");
  run<false, 0, 8>(8, "alone");
  run<true, 0, 8>(8, "alone");
  run<false, 1, 8>(16, "+8 polling waves");
  run<true, 1, 8>(16, "+8 polling waves");
  return 0;
}
