// xchg_probe — cost of one cross-wave exchange inside a workgroup on gfx950
// (development probe for the scene kernel's per-frame recurrence exchange).
// One workgroup = NW exchanging waves (one per SIMD) + optional idle waves;
// each iteration every exchanging wave writes a 4-float partial quad and its
// sequence word, then waits until all NW sequence words reach the
// iteration.  Variants:
//   0 poll: LDS sequence words, the scene kernel's poll (word + quad in one
//     round trip, ballot)
//   1 barrier: ds_write + s_barrier (only the NW waves in the workgroup)
//   2 poll, data-as-flag: the partials carry the iteration in a second dword
//     (ds_write_b64 {value, iter}); no separate sequence word
// Prints cycles per iteration (s_memtime of wave 0, median over workgroups).
// build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/xchg_probe tools/probes/xchg_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kIters = 256;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int VAR, int NW>
__global__ void __launch_bounds__(1024) xchg(unsigned long long* out, int nwaves) {
  __shared__ __attribute__((aligned(16))) float red[2][NW * 16];
  __shared__ __attribute__((aligned(16))) int seq[NW];
  __shared__ __attribute__((aligned(16))) float red2[2][NW * 16 * 2];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, L = lane & 15, q = lane >> 4;
  if (threadIdx.x < NW) seq[threadIdx.x] = 0;
  for (int i = threadIdx.x; i < 2 * NW * 32; i += blockDim.x) (&red2[0][0])[i] = -1.f;
  __syncthreads();
  if (wv >= NW) return;   // idle waves leave
  float acc = 1.f + lane;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
    const int b = it & 1;
    if (VAR == 0) {
      if (L < 4) red[b][wv * 16 + 4 * q + L] = acc;
      asm volatile("" ::: "memory");
      if (lane == 0) asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(seq + wv)), "v"(it + 1) : "memory");
      int sq;
      float4 r;
      const uint32_t sa = lds_addr(seq + (L & 3)), ra = lds_addr(&red[b][(L & 3) * 16 + 4 * q]);
      for (;;) {
        asm volatile("ds_read_b32 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(sq), "=&v"(r) : "v"(sa), "v"(ra) : "memory");
        if (__builtin_amdgcn_ballot_w64(sq < it + 1) == 0) break;
      }
      acc += r.x * 1e-9f;
    } else if (VAR == 1) {
      if (L < 4) red[b][wv * 16 + 4 * q + L] = acc;
      __syncthreads();
      const float4 r = *reinterpret_cast<const float4*>(&red[b][(L & 3) * 16 + 4 * q]);
      acc += r.x * 1e-9f;
    } else {
      // {value, iteration} pairs: the reader checks the iteration of every pair it reads
      if (L < 4) {
        const uint32_t wa = lds_addr(&red2[b][(wv * 16 + 4 * q + L) * 2]);
        asm volatile("ds_write_b64 %0, %1" ::"v"(wa), "v"(make_float2(acc, __int_as_float(it + 1))) : "memory");
      }
      const uint32_t ra = lds_addr(&red2[b][((L & 3) * 16 + 4 * q) * 2]);
      float4 r0, r1;
      for (;;) {
        asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(r0), "=&v"(r1) : "v"(ra) : "memory");
        const int m = min(min(__float_as_int(r0.y), __float_as_int(r0.w)),
                          min(__float_as_int(r1.y), __float_as_int(r1.w)));
        if (__builtin_amdgcn_ballot_w64(m < it + 1) == 0) break;
      }
      acc += r0.x * 1e-9f;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0;
  if (acc == 12345.f) out[0] = 0;
}

template <int VAR>
void run(int nblocks, int nwaves, const char* name) {
  unsigned long long* d;
  hipMalloc(&d, nblocks * sizeof(unsigned long long));
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((xchg<VAR, 4>), dim3(nblocks), dim3(64 * nwaves), 0, 0, d, nwaves);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(nblocks);
  hipMemcpy(h.data(), d, nblocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  printf("%-22s blocks %4d waves %2d: %.1f cycles per exchange (median), max %.1f\n", name, nblocks, nwaves,
         (double)h[nblocks / 2] / kIters, (double)h.back() / kIters);
  hipFree(d);
}

int main() {
  for (int nb : {1, 256}) {
    run<0>(nb, 4, "poll (seq + quad)");
    run<1>(nb, 4, "s_barrier");
    run<2>(nb, 4, "poll (value+iter)");
  }
  return 0;
}
