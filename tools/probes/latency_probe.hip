// Diagnostic probe (not part of the product): per-workgroup latency of the
// first global loads at kernel start, 256 workgroups, each touching its own
// region of a buffer (s_memtime ticks), and of a 4-byte LDS-DMA batch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void __launch_bounds__(256) probe(const float* __restrict__ buf, size_t stride_floats,
                                             unsigned long long* out, float* sink, int mode) {
  __shared__ float lds[4096];
  const int b = blockIdx.x, t = threadIdx.x;
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  float v = 0.f;
  const float* p = buf + (size_t)b * stride_floats;
  if (mode == 0) {                       // one dword per lane
    v = p[t];
  } else if (mode == 1) {                // 4 KB per workgroup by 4-byte LDS-DMA
    for (int i = (t >> 6) * 64; i < 1024; i += 256)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p + i + (t & 63)),
                                       (__attribute__((address_space(3))) void*)(lds + i), 4, 0, 0);
  } else {                               // 16 KB per workgroup, float4 loads
    const float4* p4 = reinterpret_cast<const float4*>(p);
    float4 a = p4[t], c = p4[t + 256], d = p4[t + 512], e = p4[t + 768];
    v = a.x + c.y + d.z + e.w;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  if (t == 0) out[b] = t1 - t0;
  if (v == 12345.f) sink[b] = v + lds[t];
}

int main() {
  const int nb = 256;
  const size_t stride = 64 * 1024;       // 256 KB apart
  float* buf; unsigned long long* out; float* sink;
  hipMalloc(&buf, nb * stride * sizeof(float));
  hipMemset(buf, 0, nb * stride * sizeof(float));
  hipMalloc(&out, nb * sizeof(unsigned long long));
  hipMalloc(&sink, nb * sizeof(float));
  std::vector<unsigned long long> h(nb);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 4; ++rep) {
      hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 0, 0, buf, stride, out, sink, mode);
      hipDeviceSynchronize();
      hipMemcpy(h.data(), out, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost);
      unsigned long long mn = ~0ull, mx = 0, sum = 0;
      for (auto x : h) { mn = x < mn ? x : mn; mx = x > mx ? x : mx; sum += x; }
      printf("mode %d rep %d: ticks min %llu mean %llu max %llu\n", mode, rep, mn, sum / nb, mx);
    }
  }
  return 0;
}
