// rows_probe — what bounds the train step's row sum (g2k_grad_rows_kernel:
// grad[p] = sum over S scene rows, fixed order) on gfx950.  A writer kernel
// stands in for the scene kernel (one workgroup per scene writes its row),
// then one of the row-sum variants below reads the S x width rows; run under
// rocprofv3 --kernel-trace --stats for each kernel's average duration.
//   V0  32 columns x 32 row slices (1024 threads), 8 rows per thread in
//       flight (the kernel's current shape)
//   V1  64 columns x 16 slices (1024 threads), 16 rows per thread in flight
//   V2  32 columns x 8 slices (256 threads), 32 rows per thread in flight
//   V3  float4 columns: 8 column quads x 32 slices (256 threads), 8 rows
//   V4  float4 columns: 16 column quads x 16 slices (256 threads), 16 rows
//   V9  floor: every thread loads one float and stores it
// build: hipcc --offload-arch=gfx950 -O3 -o tools/probes/rows_probe tools/probes/rows_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ void writer(float* rows, int width, int iter) {
  float* r = rows + (size_t)blockIdx.x * width;
  for (int p = threadIdx.x; p < width; p += blockDim.x) r[p] = (float)((p + blockIdx.x + iter) & 15);
}

// COLS x SLICES threads; thread (c, sl) sums rows sl, sl + SLICES, ... of column
// blockIdx.x * COLS + c with RIF rows per round in flight, then the slices in order
template <int COLS, int SLICES, int RIF>
__global__ void __launch_bounds__(COLS * SLICES) rows_scalar(const float* __restrict__ rows, int S,
                                                             int width, float* __restrict__ grad) {
  __shared__ float red[SLICES][COLS + 1];
  const int c = threadIdx.x % COLS, sl = threadIdx.x / COLS;
  const int p = blockIdx.x * COLS + c;
  float acc = 0.f;
  if (p < width) {
    for (int r0 = sl; r0 < S; r0 += RIF * SLICES) {
      float v[RIF];
#pragma unroll
      for (int i = 0; i < RIF; ++i) {
        const int r = r0 + i * SLICES;
        v[i] = rows[(size_t)(r < S ? r : S - 1) * width + p];
      }
#pragma unroll
      for (int i = 0; i < RIF; ++i) acc += r0 + i * SLICES < S ? v[i] : 0.f;
    }
  }
  red[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && p < width) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < SLICES; ++k) t += red[k][c];
    grad[p] = t;
  }
}

// QUADS x SLICES threads, float4 columns (width a multiple of 4 here)
template <int QUADS, int SLICES, int RIF>
__global__ void __launch_bounds__(QUADS * SLICES) rows_quad(const float* __restrict__ rows, int S,
                                                            int width, float* __restrict__ grad) {
  __shared__ float4 red[SLICES][QUADS];
  const int c = threadIdx.x % QUADS, sl = threadIdx.x / QUADS;
  const int p = 4 * (blockIdx.x * QUADS + c);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (p < width) {
    for (int r0 = sl; r0 < S; r0 += RIF * SLICES) {
      float4 v[RIF];
#pragma unroll
      for (int i = 0; i < RIF; ++i) {
        const int r = r0 + i * SLICES;
        v[i] = *reinterpret_cast<const float4*>(rows + (size_t)(r < S ? r : S - 1) * width + p);
      }
#pragma unroll
      for (int i = 0; i < RIF; ++i) {
        const float m = r0 + i * SLICES < S ? 1.f : 0.f;
        acc.x = fmaf(m, v[i].x, acc.x); acc.y = fmaf(m, v[i].y, acc.y);
        acc.z = fmaf(m, v[i].z, acc.z); acc.w = fmaf(m, v[i].w, acc.w);
      }
    }
  }
  red[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && p < width) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < SLICES; ++k) {
      t.x += red[k][c].x; t.y += red[k][c].y; t.z += red[k][c].z; t.w += red[k][c].w;
    }
    *reinterpret_cast<float4*>(grad + p) = t;
  }
}

__global__ void floor_kernel(const float* __restrict__ rows, int width, float* __restrict__ grad) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p < width) grad[p] = rows[p];
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? std::atoi(argv[1]) : 256;
  const int width = argc > 2 ? std::atoi(argv[2]) : 1268;     // P + 2 rounded to a quad
  const int reps = 200;
  float *rows, *grad;
  CK(hipMalloc(&rows, (size_t)S * width * 4));
  CK(hipMalloc(&grad, (size_t)width * 4 * 8));
  std::vector<float> ref(width), got(width);
  auto check = [&](const char* name, int v) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), grad + (size_t)v * width, width * 4, hipMemcpyDeviceToHost));
    double err = 0;
    for (int p = 0; p < width; ++p) err = std::max(err, (double)std::abs(got[p] - ref[p]));
    std::printf("%s max abs err %.3g\n", name, err);
  };
  // reference sums of the last writer iteration
  for (int p = 0; p < width; ++p) {
    double t = 0;
    for (int s = 0; s < S; ++s) t += (float)((p + s + reps - 1) & 15);
    ref[p] = (float)t;
  }
  for (int it = 0; it < reps; ++it) {
    // the writer before every variant: each reads rows fresh from another kernel
    auto W = [&] { hipLaunchKernelGGL(writer, dim3(S), dim3(256), 0, 0, rows, width, it); };
    W(); hipLaunchKernelGGL((rows_scalar<32, 32, 8>), dim3((width + 31) / 32), dim3(1024), 0, 0, rows, S, width, grad);
    W(); hipLaunchKernelGGL((rows_scalar<64, 16, 16>), dim3((width + 63) / 64), dim3(1024), 0, 0, rows, S, width, grad + width);
    W(); hipLaunchKernelGGL((rows_scalar<32, 8, 32>), dim3((width + 31) / 32), dim3(256), 0, 0, rows, S, width, grad + 2 * width);
    W(); hipLaunchKernelGGL((rows_quad<8, 32, 8>), dim3((width / 4 + 7) / 8), dim3(256), 0, 0, rows, S, width, grad + 3 * width);
    W(); hipLaunchKernelGGL((rows_quad<16, 16, 16>), dim3((width / 4 + 15) / 16), dim3(256), 0, 0, rows, S, width, grad + 4 * width);
    W(); hipLaunchKernelGGL(floor_kernel, dim3((width + 255) / 256), dim3(256), 0, 0, rows, width, grad + 5 * width);
  }
  CK(hipGetLastError());
  check("V0 32x32x8", 0);
  check("V1 64x16x16", 1);
  check("V2 32x8x32", 2);
  check("V3 q8x32x8", 3);
  check("V4 q16x16x16", 4);
  CK(hipFree(rows));
  CK(hipFree(grad));
  return 0;
}
