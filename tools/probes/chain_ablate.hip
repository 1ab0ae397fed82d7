// chain_ablate — which part of one recurrence frame (RecurH::step_seq and
// the poll_red exchange) holds the chain: the frame loop of chain_probe with
// parts switched off one at a time (timing only; results are meaningless).
// Development probe, not product code.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I multimodaltraj_2_amd/csrc
//          -o tools/probes/chain_ablate tools/probes/chain_ablate.hip
#include <algorithm>
#include <cstdio>
#include <vector>
#include "g2k_recur.h"

using namespace g2k;

constexpr int kF = 64;
constexpr int kRB = 64;
constexpr int TPW = 2;

enum : int {
  NO_XCHG = 1,     // no waiting: read the own wave's quad once
  NO_SPLIT = 2,    // keep the B operands of the last frame
  NO_EXP = 4,      // e = acc (no v_exp)
  NO_MFMA = 8,     // acc = a (no MFMA)
  NO_REDUCE = 16,  // publish p[0] without the row reduction
  NO_APREP = 32,   // A operand = b (no z, rcp, split of A)
  NO_PF = 64,      // no As prefetch reads
};

template <int OFF>
__global__ void __launch_bounds__(256) chain(unsigned long long* out, float* hout) {
  __shared__ __attribute__((aligned(16))) float sAs[kF * 256];
  __shared__ __attribute__((aligned(16))) float sRed[4 * kRB];
  __shared__ int sFlag[kF];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, L = lane & 15, q = lane >> 4;
  for (int i = threadIdx.x; i < kF * 256; i += blockDim.x) sAs[i] = kLog2e / 16.f;
  for (int i = threadIdx.x; i < kF; i += blockDim.x) sFlag[i] = i + 1;
  int* seq = reinterpret_cast<int*>(sRed + 2 * kRB);
  if (threadIdx.x < 4) seq[threadIdx.x] = 2;
  for (int i = threadIdx.x; i < 2 * kRB; i += blockDim.x) sRed[i] = 1.f;
  __syncthreads();
  __builtin_amdgcn_s_setprio(2);
  f16x8 bo[TPW], bs[TPW];
  float x[TPW][4];
  for (int t = 0; t < TPW; ++t)
    for (int j = 0; j < 8; ++j) { bo[t][j] = (_Float16)(0.01f * j); bs[t][j] = (_Float16)(0.001f * j); }
  const float* as_lane = sAs + L * 16 + 4 * q;
  float4 b = *reinterpret_cast<const float4*>(as_lane);
  int flq = 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int g = 0; g < kF; ++g) {
    f32x4 zq;
    if (OFF & NO_XCHG) {
      asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(zq)
                   : "v"(lds_addr(sRed + (g & 1) * kRB + wv * 16 + 4 * q)) : "memory");
    } else {
      poll_red(seq + (L & 3), g + 2, sRed + (g & 1) * kRB + (L & 3) * 16 + 4 * q, zq);
    }
    if (__builtin_amdgcn_readfirstlane(flq) != g + 1) wait_as(sFlag + g, g + 1, as_lane + g * 256, b);
    const int fn = g + 1 < kF ? g + 1 : g;
    int fl = g + 2;
    f32x4 v = {b.x, b.y, b.z, b.w};
    if (!(OFF & NO_PF))
      asm volatile("ds_read_b32 %0, %2\n\tds_read_b128 %1, %3"
                   : "=&v"(fl), "=&v"(v)
                   : "v"(lds_addr(sFlag + fn)), "v"(lds_addr(as_lane + fn * 256))
                   : "memory");
    f16x8 A;
    float a0, a1, a2, a3;
    if (OFF & NO_APREP) {
      a0 = b.x; a1 = b.y; a2 = b.z; a3 = b.w;
      for (int j = 0; j < 8; ++j) A[j] = (_Float16)b.x;
    } else {
      float z[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t = zq[i];
        t += dpp<0xB1>(t);
        t += dpp<0x4E>(t);
        z[i] = t;
      }
      a0 = b.x * rcp(z[0]); a1 = b.y * rcp(z[1]); a2 = b.z * rcp(z[2]); a3 = b.w * rcp(z[3]);
      A = __builtin_bit_cast(f16x8, split4(a0, a1, a2, a3));
    }
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc[TPW];
    if (OFF & NO_MFMA) {
      for (int t = 0; t < TPW; ++t) acc[t] = f32x4{a0, a1, a2, a3 + t};
    } else {
#pragma unroll
      for (int t = 0; t < TPW; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, bo[t], f32x4{-kOff, -kOff, -kOff, -kOff}, 0, 0, 0);
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, bs[t], acc[t], 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fl), "+v"(v)::"memory");
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    float e[TPW][4];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[t][i] = acc[t][i];
        e[t][i] = (OFF & NO_EXP) ? acc[t][i] : __builtin_amdgcn_exp2f(acc[t][i]);
        p[i] += e[t][i];
      }
    float* red = sRed + ((g + 1) & 1) * kRB;
    if (OFF & NO_REDUCE) {
      if (L < 4) red[wv * 16 + 4 * q + L] = p[L & 3] + p[0];
    } else {
      const float r = reduce4_rows16<false>(p[0], p[1], p[2], p[3], L);
      if (L < 4) red[wv * 16 + 4 * q + reduce4_row(L)] = r;
    }
    asm volatile("" ::: "memory");
    if (lane == 0) lds_store_flag(seq + wv, g + 3);
    if (!(OFF & NO_SPLIT)) {
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        bo[t] = __builtin_bit_cast(f16x8, split4(e[t][0], e[t][1], e[t][2], e[t][3]));
#pragma unroll
        for (int j = 0; j < 4; ++j) { bs[t][j] = bo[t][4 + j]; bs[t][4 + j] = bo[t][j]; }
      }
    }
    flq = fl;
    b = make_float4(v[0], v[1], v[2], v[3]);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  for (int t = 0; t < TPW; ++t)
    for (int i = 0; i < 4; ++i) sum += x[t][i] + (float)bo[t][i] + (float)bs[t][i];
  hout[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
}

template <int OFF>
void run(const char* name) {
  const int nb = 256;
  unsigned long long* d;
  float* h;
  hipMalloc(&d, nb * sizeof(unsigned long long));
  hipMalloc(&h, (size_t)nb * 256 * 4);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL((chain<OFF>), dim3(nb), dim3(256), 0, 0, d, h);
  hipDeviceSynchronize();
  std::vector<unsigned long long> v(nb);
  hipMemcpy(v.data(), d, nb * 8, hipMemcpyDeviceToHost);
  std::sort(v.begin(), v.end());
  printf("%-34s %5.0f cycles per frame (median), max %5.0f\n", name, (double)v[nb / 2] / kF,
         (double)v.back() / kF);
  hipFree(d);
  hipFree(h);
}

int main() {
  run<0>("full");
  run<NO_XCHG>("no exchange wait");
  run<NO_SPLIT>("no B split");
  run<NO_EXP>("no exp");
  run<NO_MFMA>("no MFMA");
  run<NO_REDUCE>("no row reduction");
  run<NO_APREP>("no A prep");
  run<NO_PF>("no As prefetch");
  run<NO_XCHG | NO_SPLIT | NO_EXP | NO_MFMA | NO_REDUCE | NO_APREP | NO_PF>("all off (loop + publish)");
  run<NO_SPLIT | NO_EXP | NO_MFMA | NO_REDUCE | NO_APREP | NO_PF>("exchange only");
  run<NO_XCHG | NO_SPLIT | NO_REDUCE | NO_PF>("compute chain only (A, MFMA, exp)");
  return 0;
}
