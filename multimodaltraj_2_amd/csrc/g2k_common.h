// g2k_common.h — shared constants, wave-level helpers and host launcher
// declarations of the gfx950 (CDNA4) implementation of the g2k_lstm_mcr
// per-frame path.  Included by every .hip
// translation unit of libg2k_hip.so; the C ABI is in g2k_abi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "g2k_hip.h"

namespace g2k {

constexpr int kT = 8;     // obs_len (argParser.py:26-28)
constexpr int kL = 12;    // pred_len (models/g2k_lstm_mcr.py:124)
constexpr int kL2 = 24;   // 2 * pred_len rows of temp_path
constexpr int kD = 16;    // hidden_len = neighborhood_size / grid_size (train.py:93)
constexpr int kNT = 256;  // threads per workgroup (generic kernels)
constexpr int kMaxN = 256;

// last-error plumbing (g2k_abi.hip)
int set_err(int code, const char* fmt, ...);
int check_launch(const char* what);

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float rcp(float x) { return __builtin_amdgcn_rcpf(x); }

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

// The wave's index in its workgroup, provably wave-uniform (an SGPR): role
// branches, per-wave loops and s_setprio guards on it compile to scalar
// branches instead of exec-masked code.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }


// Range-checked buffer access (raw buffer resource, stride 0): a lane whose
// byte offset is >= num_records stores nothing / loads zeros.  Per-lane
// predication without a branch around the memory instruction, so the
// compiler's vmcnt bookkeeping stays exact (a store under an exec branch
// makes every later wait conservative: vmcnt(0), i.e. wait for the stores).
typedef __amdgpu_buffer_rsrc_t brsrc;
constexpr int kBufOff = 0x7ffffff0;          // an offset no buffer here reaches
__device__ __forceinline__ brsrc make_brsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
// Cache policy of the kernels' output stores: sc1 (gfx950 CPol bits: sc0 1,
// nt 2, sc1 16) — written through to the coherence point as they are made,
// so the end-of-kernel release has no dirty L2 lines of ours to write back
// (a whole launch's pred left in the XCDs' L2s cost ~1.3 us of write-back
// per step at eth_hotel_synth: 16.75 -> 15.42 us with sc1).
constexpr int kStoreAux = 16;
// the same for a plain float store (a relaxed agent-scope atomic store is a
// global_store ... sc1)
__device__ __forceinline__ void store_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void bstore(brsrc r, int off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, kStoreAux);
}
__device__ __forceinline__ void bstore4(brsrc r, int off, float a, float b, float c, float d) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kStoreAux);
}
__device__ __forceinline__ float4 bload4(brsrc r, int off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                     __uint_as_float(v[3]));
}
__device__ __forceinline__ float2 bload2(brsrc r, int off) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  return make_float2(__uint_as_float(v[0]), __uint_as_float(v[1]));
}

// LDS-DMA: 16 bytes per lane, LDS destination = wave-uniform base + 16*lane.
__device__ __forceinline__ void dma16(const float* gsrc, float* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gsrc,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0,
                                   0);
}

// Copy n4 float4s (contiguous, 16-B aligned) global -> LDS with a workgroup
// of NT threads; the caller waits (vmcnt(0)) and barriers before reading.
template <int NT>
__device__ __forceinline__ void dma_copy_n(const float* g, float* lds, int n4, int wv, int lane) {
  for (int i = wv * 64; i < n4; i += NT) {
    if (i + lane < n4) dma16(g + (size_t)(i + lane) * 4, lds + i * 4);
  }
}

// Copy n floats global -> LDS with the whole workgroup by 4-byte LDS-DMA
// (no alignment requirement beyond 4 bytes); caller waits vmcnt(0) + barrier.
template <int NT>
__device__ __forceinline__ void dma4_copy_t(const float* g, float* lds, int n, int wv, int lane) {
  for (int i = wv * 64; i < n; i += NT) {
    if (i + lane < n)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + i + lane),
                                       (__attribute__((address_space(3))) void*)(lds + i), 4, 0, 0);
  }
}

// ---------------------------------------------------------------------------
// wave-level helpers
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Sum over the 16 lanes of a DPP row; every lane of the row gets the result.
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror
  v += dpp<0x140>(v);  // row_mirror
  return v;
}


// Sum over the four 16-lane rows of a wave (lanes r, r+16, r+32, r+48),
// identical bits in all four lanes: v_permlane32_swap + v_permlane16_swap.
__device__ __forceinline__ float sum_rows4(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  auto b = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Partner lane's value across lane groups (q ^ 1 by permlane16, q ^ 2 by
// permlane32): of the pair a swap returns, one element is this lane's own
// value, the other the partner's.
__device__ __forceinline__ float partner16(float v) {
  auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return a[0] == __float_as_uint(v) ? __uint_as_float(a[1]) : __uint_as_float(a[0]);
}
__device__ __forceinline__ float partner32(float v) {
  auto a = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return a[0] == __float_as_uint(v) ? __uint_as_float(a[1]) : __uint_as_float(a[0]);
}

// Sum over all 64 lanes (DPP + permlane, no LDS); every lane gets the result.
__device__ __forceinline__ float wave_sum(float v) { return sum_rows4(row16_sum(v)); }

// Four per-lane values v[i] (rows 4q + i of an MFMA result, this lane's
// column) reduced over the 16 lanes of each lane group by a transposing
// butterfly: 2 + 1 DPP exchanges hand each lane one row, 2 more finish the
// row.  Lane L ends with the reduction of row 4q + reduce4_row(L).
__device__ __forceinline__ int reduce4_row(int L) { return 2 * (L & 1) + ((L >> 1) & 1); }

template <bool MAX>
__device__ __forceinline__ float reduce4_rows16(float v0, float v1, float v2, float v3, int L) {
  auto op = [](float x, float y) { return MAX ? fmaxf(x, y) : x + y; };
  const bool odd = (L & 1) != 0, b1 = (L & 2) != 0;
  const float s0 = odd ? v0 : v2, s1 = odd ? v1 : v3;        // rows the xor-1 partner keeps
  const float a0 = op(odd ? v2 : v0, dpp<0xB1>(s0));        // quad_perm [1,0,3,2]
  const float a1 = op(odd ? v3 : v1, dpp<0xB1>(s1));
  float r = op(b1 ? a1 : a0, dpp<0x4E>(b1 ? a0 : a1));      // quad_perm [2,3,0,1]
  r = op(r, dpp<0x124>(r));                                 // row_ror:4
  r = op(r, dpp<0x128>(r));                                 // row_ror:8
  return r;
}

// ---------------------------------------------------------------------------
// a9 error terms for one (frame, pedestrian): y = pred_path_band[:, n] as 24
// rows (x rows 0..11, y rows 12..23), tgt = 12 (x, y) pairs (16-B aligned).
// train.py:640-656: ade_i = ||P_[i][:L] - tgt[:L]||_2 (spectral) / 12,
//                   err = P_[i][L-1] - tgt[L-1]  (fde vector).
// acc: {ade_spec, count, |fde|^2, ade_l2, |fde|}
// ---------------------------------------------------------------------------
__device__ __forceinline__ void error_terms(const float* y, const float* tgt, float acc[5]) {
  const float4* t4 = reinterpret_cast<const float4*>(tgt);
  float tv[kL2];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    float4 v = t4[k];
    tv[4 * k + 0] = v.x; tv[4 * k + 1] = v.y; tv[4 * k + 2] = v.z; tv[4 * k + 3] = v.w;
  }
  float a = 0.f, b = 0.f, c = 0.f, l2 = 0.f;
  float fx = 0.f, fy = 0.f;
#pragma unroll
  for (int l = 0; l < kL; ++l) {
    const float dx = y[l] - tv[2 * l];
    const float dy = y[kL + l] - tv[2 * l + 1];
    a = fmaf(dx, dx, a);
    b = fmaf(dx, dy, b);
    c = fmaf(dy, dy, c);
    l2 += sqrtf(fmaf(dx, dx, dy * dy));
    fx = dx; fy = dy;
  }
  // largest singular value of the [L, 2] difference: sqrt(lambda_max(M^T M))
  const float hm = 0.5f * (a - c);
  const float lam = 0.5f * (a + c) + sqrtf(fmaf(hm, hm, b * b));
  const float fsq = fmaf(fx, fx, fy * fy);
  acc[0] += sqrtf(fmaxf(lam, 0.f)) * (1.0f / 12.0f);
  acc[1] += 1.0f;
  acc[2] += fsq;
  acc[3] += l2 * (1.0f / 12.0f);
  acc[4] += sqrtf(fsq);
}

// ---------------------------------------------------------------------------
// LDS polling for the wave-specialised scene kernel.  The loads are inline
// asm (the compiler may neither hoist nor merge them) and wait for their own
// data; LDS services one CU's requests in order, so a flag read that sees a
// producer's flag write is followed by data reads that see the data the
// producer wrote before it (the producer waits lgkmcnt(0) between the two).
// A poll gives up after kPollMax rounds (~50 ms) so that a broken invariant
// yields wrong numbers, not a hung GPU.
// ---------------------------------------------------------------------------
constexpr int kPollMax = 1 << 20;
__device__ __forceinline__ void poll_pause() { __builtin_amdgcn_s_sleep(1); }

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// Flag / sequence-word store: a plain ds_write_b32 (a volatile store through a
// generic pointer compiles to a flat store + vmcnt(0) wait, hundreds of cycles
// on the critical path).  Ordered after the caller's earlier LDS writes by the
// in-order LDS queue; the memory clobber keeps the compiler from sinking them.
__device__ __forceinline__ void lds_store_flag(int* p, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}



// The recurrence's per-frame exchange, split in two LDS round trips so that
// the one on the critical path is small:
//  - read_as: the producer's flag of a frame's As tile, then the lane's As
//    row quad (As[L][4q..4q+3]), one asm block (LDS serves a CU's requests in
//    order and the producer stores the tile before the flag, so a current
//    flag means a current quad).  Issued right after the previous frame's
//    publish, while the other waves are still finishing theirs.
//  - poll_red: spin on ONE wave's sequence word (lane L reads wave L & 3's:
//    seq[w] = frames whose partials w has published, +1) together with that
//    wave's row-partial quad of rows 4q..4q+3 (raw: the four waves' quads
//    are summed across each lane quad by DPP where Recur::body needs them).
//    Data is stored before the word and read after it, so a current word
//    means current data.
// Busy poll for the first rounds, then s_sleep.
__device__ __forceinline__ int read_as(const int* flag, const float* asrc, float4& b) {
  const uint32_t fa = lds_addr(flag), da = lds_addr(asrc);
  int fl;
  f32x4 v;
  asm volatile(
      "ds_read_b32 %0, %2\n\t"
      "ds_read_b128 %1, %3\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(fl), "=&v"(v)
      : "v"(fa), "v"(da)
      : "memory");
  b = make_float4(v[0], v[1], v[2], v[3]);
  return __builtin_amdgcn_readfirstlane(fl);
}

// Slow path of read_as: the tile was not ready when first read.
__device__ __forceinline__ void wait_as(const int* flag, int want, const float* asrc, float4& b) {
  for (int it = 0; it < kPollMax; ++it) {
    if (read_as(flag, asrc, b) == want) break;
    if (it >= 8) __builtin_amdgcn_s_sleep(1);   // long waits (the first heads): back off
  }
}

__device__ __forceinline__ void poll_red(const int* seq_w, int want_seq, const float* rslot,
                                         f32x4& r) {
  const uint32_t sa = lds_addr(seq_w), ra = lds_addr(rslot);
  int sq;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile(
        "ds_read_b32 %0, %2\n\t"
        "ds_read_b128 %1, %3\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(sq), "=&v"(r)
        : "v"(sa), "v"(ra)
        : "memory");
    if (__builtin_amdgcn_ballot_w64(sq < want_seq) == 0) break;
    if (it >= 8) __builtin_amdgcn_s_sleep(1);
  }
}

// Wait until all four recurrence waves' sequence words reach `want`.
__device__ __forceinline__ void poll_seq_all(const int* seq, int want) {
  const uint32_t sa = lds_addr(seq);
  i32x4 sq;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(sq) : "v"(sa) : "memory");
    const int mn = min(min(sq[0], sq[1]), min(sq[2], sq[3]));
    if (__builtin_amdgcn_readfirstlane(mn) >= want) break;
  }
}

// Wait until every lane's sequence word (lane L reads seq_w = seq + (L & 3))
// reaches `want`.
__device__ __forceinline__ void poll_seq(const int* seq_w, int want) {
  const uint32_t sa = lds_addr(seq_w);
  int sq;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(sq) : "v"(sa) : "memory");
    if (__builtin_amdgcn_ballot_w64(sq < want) == 0) break;
  }
}

// Wait until a frame flag reaches `want` (no data attached).
__device__ __forceinline__ void poll_flag(const int* flag, int want) {
  const uint32_t fa = lds_addr(flag);
  int fl;
  for (int it = 0; it < kPollMax; ++it) {
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(fl) : "v"(fa) : "memory");
    if (__builtin_amdgcn_readfirstlane(fl) == want) break;
    poll_pause();
  }
}

__host__ __device__ inline int rup4(int x) { return (x + 3) & ~3; }

// One int at a wave-uniform address by a scalar load (scalar cache), not
// through the CU's vector-memory pipeline; for data the kernel never writes.
__device__ __forceinline__ int sload_i32(const int32_t* p) {
  int v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
// two of them in one round trip
__device__ __forceinline__ void sload2_i32(const int32_t* p, const int32_t* q, int& u, int& v) {
  asm volatile("s_load_dword %0, %2, 0x0\n\ts_load_dword %1, %3, 0x0\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(u), "=&s"(v) : "s"(p), "s"(q) : "memory");
}

// Per-lane select written as bit operations (it compiles to v_cndmask_b32).
// Left to itself the compiler turns a chain of ternaries on the lane index
// (a switch) or a ternary between loaded values into exec-masked branches:
// several scalar instructions per case, and an LDS round trip per masked
// load.  (Not inline asm: the hazard recognizer does not see an asm VALU
// write that an MFMA then reads.)
__device__ __forceinline__ float lane_sel(bool c, float a, float b) {
  const int m = -(int)c;
  return __int_as_float((__float_as_int(a) & m) | (__float_as_int(b) & ~m));
}

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// online (max, sum-of-exp) pair combine
__device__ __forceinline__ void lse_combine(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

// ---------------------------------------------------------------------------
// host side: launch arguments and launchers of each translation unit
// ---------------------------------------------------------------------------
// One fused step (g2k_scene.hip).  grad_rows == NULL: reference mode;
// otherwise train mode, one gradient row [P + 2] per scene.  h_in == NULL:
// no recurrence (gradient only); pred / metrics NULL: not written.
struct StepArgs {
  g2k_dims d;
  g2k_weights w;
  const float* pos;
  const float* vislet;
  const float* G;
  const float* targets;
  const int32_t* n_active;
  const int32_t* n_frames;
  const uint8_t* ped_mask;
  const float* h_in;
  float* h_out;
  float* pred;
  float* metrics;
  float* A_out;
  float* cost_out;
  float lambda;
  float* grad_rows;   // [S * X][P + 2] or NULL (X = scene_split: one row per workgroup)
  int* grad_ticket;   // train step with update: zeroed by workgroup 0 for the gradient-row
                      // sum's last-workgroup count (g2k_train.hip), or NULL
  int* scene_ticket;  // X > 1: [S] workgroups of a scene done (zeroed on the stream before each launch)
  float* met_part;    // X > 1: [S][X][8] the workgroups' metric partials
};

// Workgroups per scene of the fused step (G2K_STEP_SPLIT, include/g2k_hip.h):
// the requested count, else enough to cover `cus` CUs (4 at most), never more
// than the frames to share.  Host arithmetic only: no HIP call.
constexpr int kMaxSplit = 4;
int device_cus();   // CUs of the current device (g2k_abi.hip; 256 without a device)
inline bool split_automatic(const g2k_dims& d) {
  return ((d.flags & G2K_STEP_SPLIT_MASK) >> G2K_STEP_SPLIT_SHIFT) == 0 &&
         !(d.flags & G2K_STEP_CORESIDENT);
}
// Every frame of a launch has the same inputs — stride 0 (each frame reads the
// same window rows) and one target set for every frame — so one frame's work
// stands for all (g2k_scene.hip frames_invariant).  The train kernels' form
// of it also needs the L2 loss and dWo kept per worker (Nmax <= 85:
// SceneLayout::dwo_seq == 0 at 12 gradient workers).
inline bool frames_invariant_dims(const g2k_dims& d) {
  return d.stride == 0 && (d.flags & G2K_STEP_TARGETS_SHARED) && !(d.flags & G2K_STEP_LOSS_NLL) &&
         12 * d.Nmax * 8 * 4 <= 32 * 1024;
}
inline int scene_split_cus(const g2k_dims& d, int cus) {
  int x = (d.flags & G2K_STEP_SPLIT_MASK) >> G2K_STEP_SPLIT_SHIFT;
  if (x == 0 && (d.flags & G2K_STEP_CORESIDENT)) x = 1;   // launches in flight fill the CUs
  if (x == 0 && frames_invariant_dims(d)) x = 1;          // one frame's work per chunk: nothing to share
  if (x == 0) x = d.S >= cus ? 1 : (d.S > 0 ? cus / d.S : 1);
  if (x > kMaxSplit) x = kMaxSplit;
  if (x > d.F) x = d.F;
  return x < 1 ? 1 : x;
}
// the split of `d`: explicit in the flags (every launch: step_args resolves
// an automatic request for the stream's device), or — the planning calls
// without a stream — the automatic choice for the CURRENT device
inline int scene_split(const g2k_dims& d) {
  return scene_split_cus(d, split_automatic(d) ? device_cus() : 1);
}
// split workspace: the scene tickets (one 64-byte line per 16 scenes), then the partials
inline int64_t split_ws_bytes(const g2k_dims& d) {
  const int x = scene_split(d);
  if (x <= 1) return 0;
  return (int64_t)((d.S + 15) / 16) * 64 + (int64_t)d.S * x * 8 * 4;
}
inline void split_ws_bind(StepArgs& a, void* ws) {
  if (scene_split(a.d) <= 1) { a.scene_ticket = nullptr; a.met_part = nullptr; return; }
  a.scene_ticket = static_cast<int*>(ws);
  a.met_part = reinterpret_cast<float*>(static_cast<char*>(ws) + (int64_t)((a.d.S + 15) / 16) * 64);
}
int scene_step_launch(const StepArgs& a, hipStream_t st);
int64_t scene_lds_bytes(const g2k_dims* d, bool grad);

// floats of one parameter vector (g2k_grad_size): + the NLL head [3][12]
constexpr int kNllHead = 3 * kL;
__host__ __device__ inline int grad_params(int Nmax, bool nll = false) {
  return 24 * Nmax + 496 + (nll ? kNllHead : 0);
}
__host__ __device__ inline bool loss_nll(const g2k_dims& d) { return (d.flags & G2K_STEP_LOSS_NLL) != 0; }

// g2k_train.hip
// the optimizer step folded into the gradient-row sum (run by the workgroup
// that finishes last; `ticket` zeroed by the same step's scene kernel)
struct UpdateArgs {
  float* params;
  float* ms;
  float lr, decay, clip;
  int* ticket;
};
int grad_rows_launch(const float* rows, int S, int width, float* grad, hipStream_t st,
                     const UpdateArgs* up = nullptr);
int update_launch(float* params, float* ms, const float* grad, int n, float lr, float decay,
                  float clip, hipStream_t st);

// g2k_nll.hip
int nll_launch(const g2k_dims* d, const float* pred, const float* targets, const int32_t* n_active,
               const int32_t* n_frames, const uint8_t* ped_mask, const float* head, float* rows,
               float* dpred, hipStream_t st);
int gauss_sample_launch(const g2k_dims* d, const float* pred, const float* head, uint64_t seed,
                        float* out, hipStream_t st);

// g2k_ops.hip
int recur_launch(const float* A, float* h, int S, int frames, int D, int H, hipStream_t st);
int mcr_forward_launch(const g2k_dims* d, const g2k_weights* w, const float* X, const float* Rel,
                       const float* G, const int32_t* n_active, float* A_out, float* cost_out,
                       float* pred, float lambda, hipStream_t st);
int embed_launch(const g2k_dims* d, const g2k_weights* w, const float* pos, const float* vislet,
                 const int32_t* n_active, float* X, float* Rel, hipStream_t st);
int errors_launch(const g2k_dims* d, const float* pred, const float* targets,
                  const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                  int variant, float* out, hipStream_t st);
int relation_launch(const float* adj, float* out, int64_t rows, int cols, bool softmax,
                    hipStream_t st);
int encoder_chain_launch(const g2k_dims* d, const g2k_weights* w, const float* X, const float* Rel,
                         const float* G, const int32_t* n_active, const int32_t* n_frames,
                         const float* cell_W, const float* cell_b, const float* cell_peep,
                         int feature_size, int num_units, float* Xe, float* cell_state, float* attn,
                         float* cost, float* pred, float* h, float lambda, hipStream_t st);
int gridlstm_launch(const float* in, int64_t ld_in, const float* state, int64_t ld_state,
                    const float* W, const float* b, const float* peep, float* out, float* state_out,
                    int64_t rows, int blocks, int feature_size, int num_units, hipStream_t st);
int ctx_conv_launch(const float* img, int Hh, int Ww, int C, const float* filt, int D, float lambda,
                    float* out, float* G, float* part, hipStream_t st);

}  // namespace g2k
