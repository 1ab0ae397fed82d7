// Diagnostic probe (not part of the product): cycles per frame of the hidden
// recurrence body (train.py:243-252) for H = 128 split over NW waves (TPW
// 16-column tiles per wave), to attribute the per-frame latency.
//   EX: 0 no exchange, 1 LDS sequence-word poll, 2 s_barrier
//   FL bits: 1 skip the 16-lane DPP row reduce, 2 skip exp, 4 one k-step per
//            tile, 8 log2e folded into A (v_exp_f32 direct) + tile-major MFMA
//            order, 16 split-f16 MFMA (16x16x32_f16, hi/lo pairs)
// 256 workgroups; lane 0 of each wave stamps s_memtime around the loop.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ int reduce4_row(int L) { return 2 * (L & 1) + ((L >> 1) & 1); }
__device__ __forceinline__ float reduce4_rows16(float v0, float v1, float v2, float v3, int L) {
  const bool odd = (L & 1) != 0, b1 = (L & 2) != 0;
  const float s0 = odd ? v0 : v2, s1 = odd ? v1 : v3;
  const float a0 = (odd ? v2 : v0) + dpp<0xB1>(s0);
  const float a1 = (odd ? v3 : v1) + dpp<0xB1>(s1);
  float r = (b1 ? a1 : a0) + dpp<0x4E>(b1 ? a0 : a1);
  r = r + dpp<0x124>(r);
  r = r + dpp<0x128>(r);
  return r;
}
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void lds_store_flag(int* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t split_pk(float x) {
  const float hi = __uint_as_float(__float_as_uint(x) & 0xFFFFE000u);
  auto v = __builtin_amdgcn_cvt_pkrtz(hi, x - hi);
  return *reinterpret_cast<uint32_t*>(&v);
}
__device__ __forceinline__ uint32_t dup_pk(float x) {
  auto v = __builtin_amdgcn_cvt_pkrtz(x, x);
  return *reinterpret_cast<uint32_t*>(&v);
}

constexpr int kNB = 256, kIters = 2000;

template <int EX, int FL, int TPW, int NW>
__global__ void __launch_bounds__(64 * NW) probe(const float* __restrict__ as_g, float* out,
                                                 unsigned long long* cyc, int iters) {
  __shared__ __attribute__((aligned(16))) float sAs[256];
  __shared__ __attribute__((aligned(16))) float red[2][16 * NW];
  __shared__ __attribute__((aligned(16))) int seq[NW + 4];
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = lane & 15, q = lane >> 4;
  for (int i = tid; i < 256; i += 64 * NW) sAs[i] = as_g[i];
  if (tid < NW + 4) seq[tid] = 0;
  if (tid < 16 * NW) { red[0][tid] = 32.f; red[1][tid] = 32.f; }
  __syncthreads();
  float e[TPW][4], x[TPW][4];
  for (int t = 0; t < TPW; ++t)
    for (int i = 0; i < 4; ++i) { e[t][i] = 1.0f + 0.01f * (L + t + i + q); x[t][i] = 0.f; }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int g = 0; g < iters; ++g) {
    float4 b = *reinterpret_cast<const float4*>(sAs + L * 16 + 4 * q);
    float z[4];
    const float* rc = red[g & 1];
    if (EX == 3) {
      // the scene kernel's poll_frame: seq int4, flag, As quad, 4 partial quads
      const uint32_t sa = lds_addr(seq), fa = lds_addr(seq + 4), da = lds_addr(sAs + L * 16 + 4 * q),
                     ra = lds_addr(rc + 4 * q);
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      i32x4 sq;
      int fl;
      f32x4 v, r0, r1, r2, r3;
      for (int it = 0; it < (1 << 12); ++it) {
        asm volatile(
            "ds_read_b128 %0, %7\n\t"
            "ds_read_b32 %1, %8\n\t"
            "ds_read_b128 %2, %9\n\t"
            "ds_read_b128 %3, %10\n\t"
            "ds_read_b128 %4, %10 offset:64\n\t"
            "ds_read_b128 %5, %10 offset:128\n\t"
            "ds_read_b128 %6, %10 offset:192\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&v"(sq), "=&v"(fl), "=&v"(v), "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
            : "v"(sa), "v"(fa), "v"(da), "v"(ra)
            : "memory");
        const int mn = min(min(sq[0], sq[1]), min(sq[2], sq[3]));
        if (__builtin_amdgcn_readfirstlane(mn) >= g && __builtin_amdgcn_readfirstlane(fl) == 0) break;
        if (it >= 8) __builtin_amdgcn_s_sleep(1);
      }
      z[0] = (r0[0] + r1[0]) + (r2[0] + r3[0]); z[1] = (r0[1] + r1[1]) + (r2[1] + r3[1]);
      z[2] = (r0[2] + r1[2]) + (r2[2] + r3[2]); z[3] = (r0[3] + r1[3]) + (r2[3] + r3[3]);
      b = make_float4(v[0], v[1], v[2], v[3]);
    } else if (EX == 1) {
      // lane (L, q) reads wave (L % NW)'s quad; NW > 4 waves need NW / 4 reads
      constexpr int R = NW > 4 ? NW / 4 : 1;
      f32x4 r[R];
      int sq[R];
      for (int it = 0; it < (1 << 12); ++it) {
        bool ok = true;
        for (int k = 0; k < R; ++k) {
          const int w = ((L & 3) + 4 * k) % NW;
          const uint32_t sa = lds_addr(seq + w), ra = lds_addr(rc + w * 16 + 4 * q);
          asm volatile("ds_read_b32 %0, %2\n\tds_read_b128 %1, %3"
                       : "=&v"(sq[k]), "=&v"(r[k]) : "v"(sa), "v"(ra) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        for (int k = 0; k < R; ++k) ok &= sq[k] >= g;
        if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
      }
      for (int i = 0; i < 4; ++i) {
        float t = r[0][i];
        for (int k = 1; k < R; ++k) t += r[k][i];
        if (NW >= 4) { t += dpp<0xB1>(t); t += dpp<0x4E>(t); }
        z[i] = t;
      }
    } else {
      for (int i = 0; i < 4; ++i) z[i] = 0.f;
      for (int w = 0; w < NW; ++w) {
        const float4 v = *reinterpret_cast<const float4*>(rc + w * 16 + 4 * q);
        z[0] += v.x; z[1] += v.y; z[2] += v.z; z[3] += v.w;
      }
    }
    const float bb[4] = {b.x, b.y, b.z, b.w};
    constexpr float kLog2e = 1.4426950408889634f;
    float a[4];
    for (int i = 0; i < 4; ++i) a[i] = bb[i] * __builtin_amdgcn_rcpf(z[i]) * ((FL & 8) ? kLog2e : 1.f);
    f32x4 acc[TPW];
    for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (FL & 16) {
      f16x8 Ah, Al, B[TPW];
      for (int j = 0; j < 4; ++j) {
        const float hi = __uint_as_float(__float_as_uint(a[j] * 4096.f) & 0xFFFFE000u);
        reinterpret_cast<uint32_t*>(&Ah)[j] = dup_pk(hi);
        reinterpret_cast<uint32_t*>(&Al)[j] = dup_pk(a[j] * 4096.f - hi);
      }
      for (int t = 0; t < TPW; ++t)
        for (int j = 0; j < 4; ++j) reinterpret_cast<uint32_t*>(&B[t])[j] = split_pk(e[t][j]);
      __builtin_amdgcn_sched_barrier(0);
      for (int t = 0; t < TPW; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah, B[t], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(Al, B[t], acc[t], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      for (int t = 0; t < TPW; ++t)
        for (int i = 0; i < 4; ++i) acc[t][i] *= (1.0f / 4096.f);
    } else {
      constexpr int NK = (FL & 4) ? 1 : 4;
      __builtin_amdgcn_sched_barrier(0);
      if (FL & 8) {
        for (int t = 0; t < TPW; ++t)
          for (int k = 0; k < NK; ++k) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], e[t][k], acc[t], 0, 0, 0);
      } else {
        for (int k = 0; k < NK; ++k)
          for (int t = 0; t < TPW; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[k], e[t][k], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    for (int t = 0; t < TPW; ++t)
      for (int i = 0; i < 4; ++i) {
        x[t][i] = acc[t][i];
        e[t][i] = (FL & 2) ? acc[t][i] : ((FL & 8) ? __builtin_amdgcn_exp2f(acc[t][i]) : __expf(acc[t][i]));
        p[i] += e[t][i];
      }
    float r;
    if (FL & 1) r = p[L & 3];
    else r = reduce4_rows16(p[0], p[1], p[2], p[3], L);
    float* rn = red[(g + 1) & 1];
    if (L < 4) rn[wv * 16 + 4 * q + reduce4_row(L)] = r;
    if (EX == 1 || EX == 3) {
      asm volatile("" ::: "memory");
      if (lane == 0) lds_store_flag(seq + wv, g + 1);
    } else if (EX == 2) {
      __syncthreads();
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0) cyc[blockIdx.x * NW + wv] = t1 - t0;
  if (tid == 0 && blockIdx.x == 0) cyc[kNB * 16 - 1] = (t1 - t0) * 1000 / ((r1 - r0) * 10);
  float sacc = 0.f;
  for (int t = 0; t < TPW; ++t)
    for (int i = 0; i < 4; ++i) sacc += x[t][i];
  out[blockIdx.x * 64 * NW + tid] = sacc;
}


template <int EX, int FL, int TPW, int NW>
void run(const char* name, const float* as, float* out, unsigned long long* cyc) {
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL((probe<EX, FL, TPW, NW>), dim3(kNB), dim3(64 * NW), 0, 0, as, out, cyc, kIters);
    (void)hipDeviceSynchronize();
  }
  std::vector<unsigned long long> c(kNB * NW);
  (void)hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long mhz;
  (void)hipMemcpy(&mhz, cyc + kNB * 16 - 1, 8, hipMemcpyDeviceToHost);
  std::sort(c.begin(), c.end());
  printf("%-40s cycles/frame: min %7.1f median %7.1f max %7.1f  (clock %llu MHz)\n", name, c[0] / (double)kIters,
         c[c.size() / 2] / (double)kIters, c.back() / (double)kIters, mhz);
}

int main() {
  float *as, *out;
  unsigned long long* cyc;
  (void)hipMalloc(&as, 256 * 4);
  (void)hipMalloc(&out, kNB * 1024 * 4);
  (void)hipMalloc(&cyc, kNB * 16 * 8);
  std::vector<float> h(256);
  for (int i = 0; i < 256; ++i) h[i] = 1.0f / 16 + 0.001f * (i % 7);
  (void)hipMemcpy(as, h.data(), 256 * 4, hipMemcpyHostToDevice);
  run<0, 0, 2, 4>("f32 4w no-exch", as, out, cyc);
  run<1, 0, 2, 4>("f32 4w lds-seq", as, out, cyc);
  run<1, 8, 2, 4>("f32 4w lds-seq log2e", as, out, cyc);
  run<3, 8, 2, 4>("f32 4w scene-poll log2e", as, out, cyc);
  run<3, 0, 2, 4>("f32 4w scene-poll", as, out, cyc);
  std::vector<float> o(kNB * 1024);
  (void)hipMemcpy(o.data(), out, o.size() * 4, hipMemcpyDeviceToHost);
  printf("checksum %f\n", o[0] + o[1000]);
  return 0;
}
