// FETCH_SIZE calibration probe (development tool, not product code): each
// kernel reads exactly `bytes` distinct bytes of a buffer larger than the
// 256 MiB MALL once, by one access pattern; rocprofv3 --pmc FETCH_SIZE per
// kernel divided by the known bytes gives the counter's scale for that
// pattern (the scene kernel reads by 4-byte LDS-DMA, 16-byte LDS-DMA and
// 8-byte buffer loads).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/fetch_probe tools/probes/fetch_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int kThreads = 256;

__global__ void __launch_bounds__(kThreads) probe_vec16(const float4* __restrict__ src, int64_t n4, float* out) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const float4 v = src[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[0] = acc;
}

__global__ void __launch_bounds__(kThreads) probe_buf8(const float* __restrict__ src, int64_t n2, float* out) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n2; i += (int64_t)gridDim.x * kThreads) {
    const float2 v = reinterpret_cast<const float2*>(src)[i];
    acc += v.x + v.y;
  }
  if (acc == 12345.f) out[0] = acc;
}

#define PROBE_LDS_DMA(NAME, B)                                                                      \
  __global__ void __launch_bounds__(kThreads) NAME(const float* __restrict__ src, int64_t nelem,    \
                                                   float* out) {                                   \
    /* each wave moves 64 * B bytes per instruction into its LDS slice */                          \
    __shared__ __attribute__((aligned(16))) float lds[kThreads * 4];                                \
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;                                       \
    constexpr int per = B / 4;                                                                      \
    const int64_t step = (int64_t)gridDim.x * kThreads * per;                                       \
    for (int64_t i = ((int64_t)blockIdx.x * kThreads + wv * 64) * per; i < nelem; i += step) {      \
      if (i + (int64_t)(lane + 1) * per <= nelem)                                                   \
        __builtin_amdgcn_global_load_lds(                                                           \
            (const __attribute__((address_space(1))) void*)(src + i + lane * per),                  \
            (__attribute__((address_space(3))) void*)(lds + wv * 64 * per), B, 0, 0);               \
    }                                                                                               \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                               \
    __syncthreads();                                                                                \
    if (lds[threadIdx.x] == 12345.f) out[0] = lds[threadIdx.x];                                    \
  }
PROBE_LDS_DMA(probe_lds_dma4, 4)
PROBE_LDS_DMA(probe_lds_dma16, 16)

int main(int argc, char** argv) {
  const int64_t bytes = (argc > 1 ? atoll(argv[1]) : 64ll) << 20;   // MiB per probe
  const int64_t nbuf = 6;                                           // distinct buffers: no cache reuse
  float* buf[nbuf];
  float* out;
  for (int i = 0; i < nbuf; ++i) {
    if (hipMalloc(&buf[i], bytes) != hipSuccess) return 1;
    hipMemset(buf[i], 0, bytes);
  }
  hipMalloc(&out, 64);
  // flush the MALL with a large untouched buffer's memset
  float* big;
  hipMalloc(&big, 512ll << 20);
  hipMemset(big, 1, 512ll << 20);
  hipDeviceSynchronize();
  const int grid = 256 * 8;
  probe_vec16<<<grid, kThreads>>>(reinterpret_cast<const float4*>(buf[0]), bytes / 16, out);
  probe_buf8<<<grid, kThreads>>>(buf[1], bytes / 8, out);
  probe_lds_dma4<<<grid, kThreads>>>(buf[2], bytes / 4, out);
  probe_lds_dma16<<<grid, kThreads>>>(buf[3], bytes / 4, out);
  hipDeviceSynchronize();
  printf("fetch_probe: %lld bytes per kernel (vec16, buf8, lds_dma4, lds_dma16)\n", (long long)bytes);
  return 0;
}
