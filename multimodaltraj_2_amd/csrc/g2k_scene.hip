// g2k_scene.hip — the fused per-frame step (train.py:197-276 over S scenes x
// F frames) in ONE launch, and its train mode: the same launch also forms
// the scene's loss gradient (SURVEY.md §8(d) "--mode train").
//
// g2k_scene_kernel<TPW, NP, GRAD>: one workgroup per scene, wave-specialised.
// Waves 0..3 (one per SIMD) run the frame-sequential recurrence (a8,
// Recur::step_seq, h in MFMA registers); waves 4..4+NP-1 are producers that
// run the frame-parallel body: frame heads (a2-a7: window norms, embeddings,
// E, A, As, M = Wc @ cost) into LDS rings with per-frame flags, then the
// prediction tiles (Y = M @ Wo, pred_path_band) with the a9 error terms.  The
// two roles never share a barrier inside a chunk of frames: the recurrence's
// latency chain runs while the producers stream predictions, targets and
// errors, and As never leaves the CU.
//
// GRAD (train mode): each producer owns whole frames (fl = pw, pw + NP, ...)
// and, per 16-pedestrian tile, turns the prediction error into dY (masked),
// dM_f += dY @ Wo^T and dWo^T += dY^T @ M_f; after its frame's tiles it forms
// the frame's weight-side terms (dcost = Wc^T dM, dE = lambda dcost G^T,
// dWc_f = dM cost^T, dK1_f = dE Uaug^T, dUaug_f = K1^T dE) and adds them into
// the scene's accumulators in frame order (an LDS sequence word: the same
// sums in the same order whatever the timing -> deterministic, no atomics on
// data).  After the last frame the producers expand the accumulators into
// the scene's gradient row [P + 2] (Wi through the window norms, Wii / Wv
// through K1 = Wv[:, :16] Wii) — no recomputed forward, no second read of the
// inputs except the position rows for dWi.  The rows are summed over scenes
// by g2k_grad_rows_kernel (g2k_train.hip) in a fixed order.
#include "g2k_common.h"
#include "g2k_recur.h"

namespace g2k {
namespace {

constexpr int kSceneChunk = 32;
constexpr int kRecW = 4;
constexpr int64_t kCoresidentLds = 80 * 1024;   // G2K_STEP_CORESIDENT: two workgroups' LDS per CU
// small block of weights / per-scene matrices in LDS (floats)
constexpr int SM_WII = 0;     // [16][8]
constexpr int SM_WV = 128;    // [8][18]
constexpr int SM_BV = 272;    // [16]
constexpr int SM_WR = 288;    // [8][2]
constexpr int SM_WC = 304;    // [24][8]
constexpr int SM_G = 496;     // [16][8]  G (lambda applied at use)
// weight-derived matrices (frame head): K1 = [Wv16 @ Wii | Wv[:,16] | Wv[:,17] | 1 | 0]
// ([8][12]), K2 = Wc @ K1 ([24][12]).  PAD (the forward kernels, whose LDS
// has room): stored zero-padded to the 16 lanes of an MFMA operand — K1 as
// [16][kKP] (rows 8..15 zero), K2 as [32][kKP] (x rows 0..11 at 0..11, y rows
// 12..23 at 16..27, rows 12..15 and 28..31 zero) — with lambda G as [16][kGP]
// (columns 8..15 zero), so that the frame heads load every operand straight
// (no clamped index, no select per operand).  The pitches keep those loads
// free of bank conflicts (the clamped reads they replace were broadcasts):
// 18 L mod 32 takes the 16 even residues, so the half-wave's (L, q < 2) words
// 18 L + q fall in 32 distinct banks; lambda G is read 16 bytes per lane, and
// 20 L mod 32 puts eight lanes' four-bank groups apart.  The train kernels
// keep the dense [8][12] / [24][12] form (their LDS is at the 160 KB limit).
constexpr int SM_K1 = 640;
constexpr int kKP = 18, kGP = 20;
template <bool PAD> struct SmallBlock {
  static constexpr int K2 = PAD ? SM_K1 + 16 * kKP : 752;
  static constexpr int LG = SM_K1 + 48 * kKP;      // (PAD only; 16-byte aligned)
  static constexpr int SPARE = PAD ? LG + 16 * kGP : 1084;   // write-only word (stores of lanes without an entry)
  static constexpr int size = SPARE + 4;
};
static_assert(SmallBlock<false>::size == 1088 && SmallBlock<true>::LG % 4 == 0, "small block");
constexpr int kKA = 12;       // augmented contraction length (8 window rows + Ve0, Ve1, bv, 0)
constexpr int kYP = 17;       // train: per-producer dY tile scratch [24][kYP] (pitch: bank spread)
// global stores per prediction tile: pred_path_band (4-byte path) / pedestrian-major (16-byte)
template <bool PM> constexpr int tile_stores() { return PM ? 2 : 8; }
// train mode
constexpr int kGFrame = 192;  // per-producer frame scratch: dM [24][8] (frame_grad's P6)
constexpr int kGT_DM = 0;
constexpr int kGAccFixed = 320;   // dWc [24][8], dK1 [8][10], dVe [2][16], dbv [16]
constexpr int kGA_WC = 0, kGA_K1 = 192, kGA_VE = 272, kGA_BV = 304;

struct SceneLayout {
  int fc, wcmax, pp;   // frames per chunk, window rows per chunk, pos row pitch (floats)
  int o_wi, o_wo, o_vis, o_v, o_small, o_y, o_met, o_ring, o_mring, o_flag, o_mflag, o_red,
      o_pos, o_vg, o_mask;
  // train mode (zero-sized otherwise)
  int wtot;            // window rows of the whole scene ((F - 1) * stride + T)
  int dwo_seq;         // 1: dWo^T accumulated in frame order (one copy); 0: one copy per producer
  int o_cost, o_gframe, o_gpriv, o_gpdv, o_gacc, o_gdv, o_gdwo, o_gseq;
  // train mode with the NLL loss (zero-sized otherwise): per-lane head-gradient
  // sums [NG][64][12], per-worker sums [NG][36], the head's raw values [36] and
  // its per-step constants [5][12] (1/sigma_x, 1/sigma_y, rho, 1/(1-rho^2), base)
  int o_nlla, o_nllw, o_nllr, o_nllc;
  int tfb;             // target bytes per frame (0: one set for every frame, G2K_STEP_TARGETS_SHARED)
  int split;           // workgroups per scene (scene_split): workgroup x owns the frames g = x mod split
  int total;           // floats
  int own0;            // > 0 (train, split 2): block ownership instead — workgroup 0 owns the first
                       // min(own0, cnt / 2) frames of each chunk, workgroup 1 the rest (own_frames)
};

__host__ __device__ inline SceneLayout scene_layout_fc(int Nmax, int stride, int F, int fc, int NP,
                                                       bool grad, bool nll = false, bool inv = false) {
  SceneLayout s;
  s.fc = fc;
  s.split = 1;
  s.own0 = 0;
  s.tfb = Nmax * kL2 * 4;
  s.wcmax = (fc - 1) * stride + kT;
  s.pp = 2 * Nmax;                            // unpadded: the chunk's rows are one contiguous copy
  int o = 0;
  s.o_wi = o;    o += rup4(Nmax * kD);
  s.o_wo = o;    o += rup4(kT * Nmax);
  s.o_vis = o;   o += rup4(2 * Nmax);                  // vislet rows
  s.o_mask = o;  o += rup4((Nmax + 3) / 4);            // the scene's ped_mask row (LDS-DMA, dword rows)
  const bool pad = !grad;                              // (SmallBlock<PAD>: the frame heads' operands)
  s.o_v = o;     o += pad ? (s.wcmax + 4) * kD : rup4((s.wcmax + 2) * kD);   // V rows: window, Ve0, Ve1 (PAD: bv, 0)
  s.o_small = o; o += pad ? SmallBlock<true>::size : SmallBlock<false>::size;
  const int NG = NP + kRecW;                          // train: producers + recurrence waves
  s.o_y = o;     o += grad ? NG * kL2 * kYP : 0;      // dY tile scratch (train)
  s.o_met = o;   o += (grad ? NG : NP) * 8;
  const int slots = inv ? 1 : fc;                     // (loop-invariant frames: one slot, frames_invariant)
  s.o_ring = o;  o += slots * kD * kD;
  s.o_mring = o; o += slots * kL2 * kT;               // M = Wc @ cost per frame [24][8]
  s.o_flag = o;  o += rup4(fc);                      // As ring flags (recurrence polls)
  s.o_mflag = o; o += rup4(fc);                      // M ring flags (prediction tiles poll)
  s.o_red = o;   o += 4 * 16 * kRecW;
  s.o_pos = o;   o += s.wcmax * s.pp;                  // raw position window (LDS-DMA)
  // VG = V @ g: window, Ve0, Ve1, bv rows [.][8] (PAD: [.][16], columns 8..15
  // zero, and a zero row)
  s.o_vg = o;    o += pad ? (s.wcmax + 4) * kD : rup4((s.wcmax + 3) * kT);
  s.wtot = (F > 0 ? F - 1 : 0) * stride + kT;
  s.dwo_seq = (int64_t)(NP + kRecW) * Nmax * kT * 4 > 32 * 1024 ? 1 : 0;
  s.o_cost = s.o_gframe = s.o_gpriv = s.o_gpdv = s.o_gacc = s.o_gdv = s.o_gdwo = s.o_gseq = o;
  s.o_nlla = s.o_nllw = s.o_nllr = s.o_nllc = o;
  if (grad) {
    s.o_cost = o;   o += fc * kT * kT;                 // cost_f per chunk frame (head -> terms)
    s.o_gframe = o; o += NG * kGFrame;
    s.o_gacc = o;   o += kGAccFixed;                   // (zeroed from here to the seq words)
    s.o_gpriv = o;  o += NG * kGAccFixed;              // each worker's sums of its frames' terms
    s.o_gpdv = o;   o += NG * s.wcmax * kD;            // ... and of its dU rows in the chunk
    s.o_gdv = o;    o += rup4(s.wtot * kD);            // dV: window-row gradient [wtot][16]
    s.o_gdwo = o;   o += (s.dwo_seq ? 1 : NG) * Nmax * kT;   // dWo^T [Nmax][8]
    s.o_nlla = o;   o += nll ? NG * 64 * 12 : 0;       // (zeroed with the sums above)
    s.o_nllw = o;   o += nll ? NG * kNllHead : 0;
    s.o_gseq = o;   o += rup4(2 + (Nmax + 15) / 16);   // chunk count, -, dWo tile seqs
    s.o_nllr = o;   o += nll ? kNllHead : 0;
    s.o_nllc = o;   o += nll ? 5 * kL : 0;
  }
  s.total = o;
  return s;
}

// Every frame of a scene has the same inputs: stride 0 (each frame reads the
// same window rows) and one target set for every frame
// (G2K_STEP_TARGETS_SHARED) — sample.py's time-slice scenes, the train.py
// legs.  E, A, As, cost, M, Y and the a9 terms are then the same in every
// frame and only h changes along them, so the step (g2k_scene_kernel<...,
// INV>, one workgroup per scene: the automatic split is 1) forms one head and
// one set of tiles per chunk, replicates their outputs over the chunk's frames
// and, in train mode, adds their gradient terms with weight n (the frames of
// the chunk); its rings hold one slot.
__host__ inline bool frames_invariant(const g2k_dims& d, bool grad) {
  (void)grad;   // (train mode: frames_invariant_dims also excludes the NLL loss and dwo_seq)
  return frames_invariant_dims(d) && scene_split(d) == 1;
}

__host__ inline SceneLayout scene_layout(const g2k_dims* d, int NP, bool grad) {
  const bool nll = grad && loss_nll(*d);
  const bool inv = frames_invariant(*d, grad);
  int fc = d->F < 1 ? 1 : (d->F < kSceneChunk ? d->F : kSceneChunk);
  SceneLayout l = scene_layout_fc(d->Nmax, d->stride, d->F, fc, NP, grad, nll, inv);
  while ((int64_t)l.total * 4 > 160 * 1024 && fc > 1) {
    fc = (fc + 1) / 2;
    l = scene_layout_fc(d->Nmax, d->stride, d->F, fc, NP, grad, nll, inv);
  }
  l.tfb = (d->flags & G2K_STEP_TARGETS_SHARED) ? 0 : d->Nmax * kL2 * 4;
  l.split = scene_split(*d);
  // train mode, two workgroups per scene: workgroup 0 also forms every frame's
  // As head for the chain (and runs the chain on its SIMDs), so it owns fewer
  // frames (M, tiles, gradient) than workgroup 1 — the modular split left it
  // ~10k cycles behind (kfold4 train, profiles/r12j_*).  One frame per
  // producer measured best: kfold4 train 41.1 -> 38.6 us per step at 8 of 20
  // frames, 42.0-42.2 at 7 or 9 (profiles/r12kl_*).  With dWo added in frame
  // order (Nmax > 85: many tiles per frame, the heads a small share) one
  // frame fewer than half: dense_crowd train 105.0 -> 101.3 us at 9 of 20
  // (8: 107.8, profiles/r12r_*, r12s_*)
  if (grad && l.split == 2 && !nll) l.own0 = l.dwo_seq ? (fc / 2 - 1 > 1 ? fc / 2 - 1 : 1) : NP;
  return l;
}

// The frames of chunk [fb, fb + cnt) a workgroup owns (global frames g with
// g mod split == x): local frames fo + split * i, i < n.  own0 > 0
// (SceneLayout::own0, split 2, the BLK kernels): blocks — workgroup 0 the
// chunk's first n0 frames, workgroup 1 the rest (local frames fo + i).
struct OwnFrames {
  int fo, n;
};
__device__ __forceinline__ int own_block0(int cnt, int own0) {
  const int h = cnt / 2;
  return own0 < h ? own0 : h;
}
__device__ __forceinline__ OwnFrames own_frames(int fb, int cnt, int split, int x, int own0) {
  if (own0 > 0) {
    const int n0 = own_block0(cnt, own0);
    return x == 0 ? OwnFrames{0, n0} : OwnFrames{n0, cnt - n0};
  }
  int fo = x - fb % split;
  if (fo < 0) fo += split;
  return OwnFrames{fo, fo < cnt ? (cnt - fo + split - 1) / split : 0};
}
// the workgroup owning local frame fl of chunk [fb, fb + cnt)
__device__ __forceinline__ int frame_owner(int fb, int cnt, int fl, int split, int own0) {
  if (own0 > 0) return fl < own_block0(cnt, own0) ? 0 : 1;
  return (fb + fl) % split;
}

// frame head output: the x / y row tiles of M^T
struct FrameHeadOut {
  f32x4 mT0, mT1;   // M[L][4q+i] (x rows), M[12+L][4q+i] (y rows)
};

// As = softmax(exp(A) / cumsum(exp(A), axis 0), axis -1)  (train.py:240) of
// one frame's A in the MFMA result layout (column L, rows 4q + i), written
// to as_dst [16][16].  The ratio exp(A_r) / sum_{k<=r} exp(A_k) is invariant
// to a per-column shift: with the column max M, e = exp(A - M) lies in (0, 1]
// and the prefix sums (in-lane, then across lane groups by permlane swaps)
// cannot overflow.  If a prefix sum underflows (the column's leading rows are
// ~87 below its max) the wave redoes the column with a running (max, sum)
// pair, which is exact for any finite A.  Then a 16-lane row softmax of
// values in (0, 1].  Stored as As * log2(e): the recurrence's A operand.
__device__ __forceinline__ void attn_weights(const f32x4 aA, float* as_dst, int L, int q) {
  float mx = fmaxf(fmaxf(aA[0], aA[1]), fmaxf(aA[2], aA[3]));
  mx = fmaxf(mx, partner16(mx));
  mx = fmaxf(mx, partner32(mx));
  float e[4], p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __expf(aA[i] - mx);
  p[0] = e[0];
#pragma unroll
  for (int i = 1; i < 4; ++i) p[i] = p[i - 1] + e[i];
  const float t1 = partner16(p[3]), t2 = partner32(p[3]), t3 = partner32(t1);
  const float pre = ((q & 2) ? t2 + t3 : 0.f) + ((q & 1) ? t1 : 0.f);   // groups before q
  float R[4];
  bool bad = false;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float P = pre + p[i];
    bad |= !(P >= 1e-30f);
    R[i] = e[i] * rcp(P);
  }
  if (__builtin_amdgcn_ballot_w64(bad) != 0) {
    // running (max, sum exp) down the rows; exclusive prefix over the groups
    float m_i[4], s_i[4];
    float m = aA[0], sacc = 1.0f;
    m_i[0] = m; s_i[0] = sacc;
#pragma unroll
    for (int i = 1; i < 4; ++i) {
      lse_combine(m, sacc, aA[i], 1.0f);
      m_i[i] = m; s_i[i] = sacc;
    }
    const float m1 = partner16(m), s1 = partner16(sacc);
    const float m2 = partner32(m), s2 = partner32(sacc);
    const float m3 = partner32(m1), s3 = partner32(s1);
    float pm = m2, ps = s2;
    lse_combine(pm, ps, m3, s3);
    float mp = -INFINITY, sp = 0.f;
    if (q & 2) { mp = pm; sp = ps; }
    if (q & 1) {
      if (q & 2) lse_combine(mp, sp, m1, s1);
      else { mp = m1; sp = s1; }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float mr = m_i[i], sr = s_i[i];
      if (q > 0) lse_combine(mr, sr, mp, sp);
      R[i] = __expf(aA[i] - mr) * rcp(sr);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float ex = __expf(R[i]);
    as_dst[(4 * q + i) * kD + L] = ex * (rcp(row16_sum(ex)) * kLog2e);
  }
}

// frame head: the g2k_lstm_mcr forward of one frame up to M (models/
// g2k_lstm_mcr.py:99-124 with train.py:178-195), reassociated around the
// weight-derived K1 / K2 (computed once per workgroup in scene_stage):
//   E    = K1 @ Uaug      Uaug = [U (8 window rows of V); Ve0; Ve1; bv; 0]
//        = Wv[:, :16] @ (Wii @ U) + Wv[:, 16:18] @ Ve + bv          (:105, 112)
//   A    = g @ (E * Rm)                                             (:105-106)
//   cost = E @ g = K1 @ VGaug        (VGaug = Uaug @ g, rows of VG)  (:112-113)
//   M    = Wc @ cost = K2 @ VGaug                                   (:119)
// Contractions over the 12 augmented rows use k = 4 ks + q (3 k-steps);
// A contracts over t = 4q + ks (rows of E as the MFMA left them).  As goes
// to `as_dst`; cost to `cost_g` (global, krnl_mdl.cost) and / or `cost_l`
// (LDS, train mode); the x / y row tiles of M^T are returned (M[L][4q+i]).
template <bool PAD, bool REP = false>
__device__ __forceinline__ FrameHeadOut frame_head(const float* sm, const float* sV,
                                                   const float* sVG, int wrow0, int wcmax,
                                                   const float (&rm)[4], float lam, float* as_dst,
                                                   int* as_flag, int flag_val, float* A_g,
                                                   float* cost_g, float* cost_l, int L, int q,
                                                   bool want_m = true, bool want_as = true,
                                                   int nrep = 1) {
  // every operand load is unconditional and issued before the first MFMA.
  // PAD: the LDS operands are zero-padded to the 16 lanes (K1, K2, lambda G,
  // VG columns; the augmented rows Ve0, Ve1, bv, 0 of V and VG), so no lane
  // selects anything.  Otherwise clamped addresses, the lanes' selects after
  // (an exec-masked load would cost its own LDS round trip on the chain).
  using SB = SmallBlock<PAD>;
  float ka[3], ua[3], va[3], bx[3], by[3], gA[4];
  if constexpr (PAD) {
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int k = 4 * ks + q;
      ka[ks] = sm[SM_K1 + L * kKP + k];
      bx[ks] = sm[SB::K2 + L * kKP + k];
      by[ks] = sm[SB::K2 + (16 + L) * kKP + k];
      const int row = ks < 2 ? wrow0 + k : wcmax + q;   // window rows, then Ve0, Ve1, bv, 0
      ua[ks] = sV[row * kD + L];
      va[ks] = sVG[row * kD + L];
    }
    {
      const float4 g = *reinterpret_cast<const float4*>(sm + SB::LG + L * kGP + 4 * q);   // lambda g[r = L][t]
      gA[0] = g.x; gA[1] = g.y; gA[2] = g.z; gA[3] = g.w;
    }
    asm volatile("" : "+v"(ka[0]), "+v"(ka[1]), "+v"(ka[2]), "+v"(ua[0]), "+v"(ua[1]), "+v"(ua[2]),
                 "+v"(va[0]), "+v"(va[1]), "+v"(va[2]));
    asm volatile("" : "+v"(bx[0]), "+v"(bx[1]), "+v"(bx[2]), "+v"(by[0]), "+v"(by[1]), "+v"(by[2]),
                 "+v"(gA[0]), "+v"(gA[1]), "+v"(gA[2]), "+v"(gA[3]));
  } else {
    const int L7 = L & 7, Lx = L < kL ? L : 0, q2 = q < 2 ? q : 1;
    float ub;
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      const int k = 4 * ks + q;
      ka[ks] = sm[SM_K1 + L7 * kKA + k];
      bx[ks] = sm[SB::K2 + Lx * kKA + k];
      by[ks] = sm[SB::K2 + (kL + Lx) * kKA + k];
      if (ks < 2) {
        ua[ks] = sV[(wrow0 + k) * kD + L];
        va[ks] = sVG[(wrow0 + k) * kT + L7];
      } else {
        ua[ks] = sV[(wcmax + q2) * kD + L];
        va[ks] = sVG[(wcmax + (q < 3 ? q : 2)) * kT + L7];   // Ve0, Ve1, bv rows
      }
    }
    ub = sm[SM_BV + L];
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) gA[ks] = sm[SM_G + L * kT + 4 * q2 + ks];   // g[r = L][t]
    asm volatile("" : "+v"(ka[0]), "+v"(ka[1]), "+v"(ka[2]), "+v"(ua[0]), "+v"(ua[1]), "+v"(ua[2]),
                 "+v"(va[0]), "+v"(va[1]), "+v"(va[2]), "+v"(ub));
    asm volatile("" : "+v"(bx[0]), "+v"(bx[1]), "+v"(bx[2]), "+v"(by[0]), "+v"(by[1]), "+v"(by[2]),
                 "+v"(gA[0]), "+v"(gA[1]), "+v"(gA[2]), "+v"(gA[3]));
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      ka[ks] = L < kT ? ka[ks] : 0.f;
      bx[ks] = L < kL ? bx[ks] : 0.f;
      by[ks] = L < kL ? by[ks] : 0.f;
      va[ks] = L < kT ? va[ks] : 0.f;
    }
    ua[2] = q < 2 ? ua[2] : (q == 2 ? ub : 0.f);
    va[2] = q == 3 ? 0.f : va[2];
  }
  // the recurrence's operand first: E -> A -> As, the As flag; M (only the
  // prediction tiles need it) after, so its six MFMAs do not hold up As.
  // (want_as false: the frame's As comes from a recurrence wave; want_m
  // false: only As — wave-uniform)
  f32x4 aA = {0.f, 0.f, 0.f, 0.f};
  if (want_as) {
    f32x4 eN = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) eN = mfma4(ka[ks], ua[ks], eN);          // E[4q+i][L]
    float em[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) em[i] = eN[i] * rm[i];                    // rm = 0 for t >= 8
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      aA = mfma4(PAD ? gA[ks] : (q < 2 ? lam * gA[ks] : 0.f), em[ks], aA);   // A[4q+i][L]
    __builtin_amdgcn_sched_barrier(0);
    attn_weights(aA, as_dst, L, q);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");          // As stored before its flag
    if ((threadIdx.x & 63) == 0) lds_store_flag(as_flag, flag_val);
    __builtin_amdgcn_sched_barrier(0);
  }
  FrameHeadOut o;
  o.mT0 = f32x4{0.f, 0.f, 0.f, 0.f};
  o.mT1 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (want_m) {   // (wave-uniform: a frame another workgroup of the scene predicts needs no M)
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) {
      o.mT0 = mfma4(va[ks], bx[ks], o.mT0);   // M[L][4q+i]       (x rows)
      o.mT1 = mfma4(va[ks], by[ks], o.mT1);   // M[12+L][4q+i]    (y rows)
    }
  }
  if (A_g && want_as) {   // (REP: the same A for nrep consecutive frames, frames_invariant)
    if constexpr (REP) {
      for (int r = 0; r < nrep; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) A_g[r * kD * kD + (4 * q + i) * kD + L] = aA[i];
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) A_g[(4 * q + i) * kD + L] = aA[i];
    }
  }
  if (cost_g || cost_l) {
    f32x4 cC = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks) cC = mfma4(ka[ks], va[ks], cC);      // cost[4q+i][L]
    if (q < 2 && L < kT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (cost_g) {
          if constexpr (REP) {
            for (int r = 0; r < nrep; ++r) cost_g[r * kT * kT + (4 * q + i) * kT + L] = cC[i];
          } else {
            cost_g[(4 * q + i) * kT + L] = cC[i];
          }
        }
        if (cost_l) cost_l[(4 * q + i) * kT + L] = cC[i];
      }
    }
  }
  return o;
}

// Per-workgroup context of the scene kernel (LDS carve-up, scene scalars).
struct SceneCtx {
  float *sWi, *sWo, *sVis, *sV, *sm, *sMet, *sRing, *sMring, *sRed, *sPos, *sVG, *sY;
  float *sCost, *sGFrame, *sGPriv, *sGPdV, *sGAcc, *sGdV, *sGdWo;
  int* sFlag;     // As ring: global frame + 1 once the frame's As is in its slot
  int* sMflag;    // M ring: global frame + 1 once the frame's M is in its slot
  int* sTicket;   // producers' metrics ticket (after the recurrence sequence words)
  int* sGseq;     // train: [0] producers done with the chunk's frames (cumulative), [2 + t]
                  // frames added to dWo tile t (dwo_seq)
  int s, x, X, tid, lane, wv, L, q, nact, nf, ntiles, ntact;   // x: this workgroup of the scene's X
  float *sNllA, *sNllW, *sNllR, *sNllC;   // NLL loss (see SceneLayout)
};

// LDS-DMA of a chunk's position window rows (train.py:76-79 window) into
// rows of pitch lay.pp = 2 Nmax: one contiguous 16-byte-per-lane copy, or (odd
// Nmax / unaligned input) wave w issues rows w, w + waves, ... by 4 bytes
template <int NT>
__device__ __forceinline__ void scene_pos_dma(const StepArgs& a, const SceneLayout& lay,
                                              const SceneCtx& c, int fb, int cnt) {
  const int Nmax = a.d.Nmax, stride = a.d.stride;
  const int wcc = (cnt - 1) * stride + kT;
  const float* src = a.pos + ((size_t)c.s * a.d.W + fb * stride) * Nmax * 2;
  const bool wide = (Nmax & 1) == 0 && (((uintptr_t)a.pos) & 15) == 0;
  if (wide) {
    // the chunk's rows are contiguous in both places: 1-KiB instructions
    // (per-row 256-B ones were 4x the instructions through the CU's
    // vector-memory pipeline, which the whole prologue queues on)
    dma_copy_n<NT>(src, c.sPos, wcc * Nmax / 2, c.wv, c.lane);
    return;
  }
  for (int r = c.wv; r < wcc; r += NT / 64) {
    const float* g = src + (size_t)r * Nmax * 2;
    float* d = c.sPos + r * lay.pp;
    for (int i = 0; i < 2 * Nmax; i += 64)
      if (i + c.lane < 2 * Nmax)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + i + c.lane),
                                         (__attribute__((address_space(3))) void*)(d + i), 4, 0, 0);
  }
}

// One 16-row tile of the chunk's embedding rows, by MFMA (train.py:76-79,
// 167-195): local rows r = w0 + L are the window rows (r < wcc: norms
// ||pos||, formed here from the LDS window), the two vislet rows and a bv
// pseudo-row (VG only).  V^T = Wi^T @ N^T over n (k = 4 ks + q), then
// VG^T = (lambda G)^T @ V^T over d with V^T straight from the registers.
// Lane (L, q) ends with V[r][4q..4q+3] and VG[r][4q..4q+3] (q < 2).
template <bool PAD>
__device__ __forceinline__ void scene_vtile(const StepArgs& a, const SceneLayout& lay,
                                            const SceneCtx& c, int w0, int wcc) {
  // branch-free: every lane loads at clamped addresses and selects, so the
  // LDS reads of several k-steps are in flight together
  const int Nmax = a.d.Nmax, L = c.L, q = c.q, nact = c.nact;
  const int r = w0 + L;
  const bool win = r < wcc, vis = r >= wcc && r < wcc + 2, bvrow = r == wcc + 2;
  const float* prow = c.sPos + (win ? r : 0) * lay.pp;
  const float* vrow = c.sVis + (vis ? r - wcc : 0) * Nmax;
  struct Raw { float wi, px, py, v; };
  auto load = [&](int ks) {
    const int n = 4 * ks + q;
    const int nc = n < Nmax ? n : Nmax - 1;
    const float2 p = *reinterpret_cast<const float2*>(prow + 2 * nc);
    return Raw{c.sWi[nc * kD + L], p.x, p.y, vrow[nc]};           // Wi[n][d = L], pos, vislet
  };
  auto value = [&](int ks, const Raw& w) {                         // N[w0 + L][n]
    const int n = 4 * ks + q;
    const float nrm = __builtin_amdgcn_sqrtf(fmaf(w.px, w.px, w.py * w.py));
    return n < nact ? (win ? nrm : (vis ? w.v : 0.f)) : 0.f;
  };
  // k-steps in groups of four (n >= nact contribute 0): no tail loop with a
  // wait per k-step
  const int nks = ((nact + 15) / 16) * 4;
  f32x4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = {0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < nks; ks += 4) {
    Raw r0 = load(ks), r1 = load(ks + 1), r2 = load(ks + 2), r3 = load(ks + 3);
    // keep all twelve loads unconditional and in flight together
    asm volatile("" : "+v"(r0.wi), "+v"(r0.px), "+v"(r0.py), "+v"(r0.v), "+v"(r1.wi), "+v"(r1.px),
                 "+v"(r1.py), "+v"(r1.v), "+v"(r2.wi), "+v"(r2.px), "+v"(r2.py), "+v"(r2.v),
                 "+v"(r3.wi), "+v"(r3.px), "+v"(r3.py), "+v"(r3.v));
    v0 = mfma4(r0.wi, value(ks, r0), v0);                          // V[w0 + L][4q + i]
    v1 = mfma4(r1.wi, value(ks + 1, r1), v1);
    v0 = mfma4(r2.wi, value(ks + 2, r2), v0);
    v1 = mfma4(r3.wi, value(ks + 3, r3), v1);
  }
  f32x4 vt;
#pragma unroll
  for (int i = 0; i < 4; ++i) vt[i] = v0[i] + v1[i];
  float gl[4], bvv[4];
#pragma unroll
  for (int ks2 = 0; ks2 < 4; ++ks2) {
    gl[ks2] = c.sm[SM_G + (4 * q + ks2) * kT + (L & 7)];                  // g[d][t2 = L]
    bvv[ks2] = c.sm[SM_BV + 4 * q + ks2];
  }
  asm volatile("" : "+v"(gl[0]), "+v"(gl[1]), "+v"(gl[2]), "+v"(gl[3]), "+v"(bvv[0]), "+v"(bvv[1]),
               "+v"(bvv[2]), "+v"(bvv[3]));
  f32x4 vg = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks2 = 0; ks2 < 4; ++ks2)
    vg = mfma4(lane_sel(L < kT, a.lambda * gl[ks2], 0.f), lane_sel(bvrow, bvv[ks2], vt[ks2]),
               vg);                                                        // VG[w0 + L][4q + i]
  const int row = win ? r : lay.wcmax + (r - wcc);               // storage row
  if (win || vis)
    *reinterpret_cast<float4*>(c.sV + row * kD + 4 * q) = make_float4(vt[0], vt[1], vt[2], vt[3]);
  if (PAD) {
    if (win || vis || bvrow)   // (lane groups 2, 3: the zero columns 8..15)
      *reinterpret_cast<float4*>(c.sVG + row * kD + 4 * q) =
          q < 2 ? make_float4(vg[0], vg[1], vg[2], vg[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
  } else if ((win || vis || bvrow) && q < 2) {
    *reinterpret_cast<float4*>(c.sVG + row * kT + 4 * q) = make_float4(vg[0], vg[1], vg[2], vg[3]);
  }
}

// K1 = [Wv[:, :16] @ Wii | Wv[:, 16] | Wv[:, 17] | 1 | 0] ([8][12]) and
// K2 = Wc @ K1 ([24][12]) by MFMA in one wave (weights only; see frame_head).
// PAD: stored zero-padded (SmallBlock; the zero rows: scene_pad_consts).
template <bool PAD>
__device__ __forceinline__ void scene_kmats(const SceneCtx& c) {
  using SB = SmallBlock<PAD>;
  const int L = c.L, q = c.q, L7 = L & 7;
  const float* sm = c.sm;
  float av[4], bw[4];
  float wv16[4], wv17[4], wc0[4], wc1[4];
  const int q1 = q & 1;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int d = 4 * q + ks;
    av[ks] = sm[SM_WV + L7 * (kD + 2) + d];                      // Wv[t = L][d]
    bw[ks] = sm[SM_WII + d * kT + L7];                           // Wii[d][k = L]
    const int t = 4 * q1 + ks;
    wv16[ks] = sm[SM_WV + t * (kD + 2) + kD];
    wv17[ks] = sm[SM_WV + t * (kD + 2) + kD + 1];
    wc0[ks] = sm[SM_WC + L * kT + 4 * q1 + ks];                 // Wc rows 0..15
    wc1[ks] = sm[SM_WC + (16 + L7) * kT + 4 * q1 + ks];        // Wc rows 16..23
  }
  asm volatile("" : "+v"(av[0]), "+v"(av[1]), "+v"(av[2]), "+v"(av[3]), "+v"(bw[0]), "+v"(bw[1]),
               "+v"(bw[2]), "+v"(bw[3]));
  asm volatile("" : "+v"(wc0[0]), "+v"(wc0[1]), "+v"(wc0[2]), "+v"(wc0[3]), "+v"(wc1[0]),
               "+v"(wc1[1]), "+v"(wc1[2]), "+v"(wc1[3]));
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    av[ks] = L < kT ? av[ks] : 0.f;
    bw[ks] = L < kT ? bw[ks] : 0.f;
    wc0[ks] = q < 2 ? wc0[ks] : 0.f;
    wc1[ks] = (q < 2 && L < kL2 - 16) ? wc1[ks] : 0.f;
  }
  f32x4 k1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) k1 = mfma4(av[ks], bw[ks], k1);   // K1[4q + i][L]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = lane_sel(L == 8, wv16[i], k1[i]);
    v = lane_sel(L == 9, wv17[i], v);
    v = lane_sel(L == 10, 1.f, v);
    k1[i] = lane_sel(q < 2 && L < kKA - 1, v, 0.f);                // column 11: 0
  }
  f32x4 ka = {0.f, 0.f, 0.f, 0.f}, kb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    ka = mfma4(wc0[ks], k1[ks], ka);                               // K2[4q + i][L]
    kb = mfma4(wc1[ks], k1[ks], kb);                               // K2[16 + 4q + i][L]
  }
  // unconditional stores: lanes without an entry write the spare word.  PAD:
  // K1 rows 8..15 are the zeros of lane groups 2, 3; K2 row r goes to r (x
  // rows, r < 12) or r + 4 (y rows)
  if constexpr (!PAD) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 4 * q + i;
      c.sm[L < kKA && q < 2 ? SM_K1 + t * kKA + L : SB::SPARE] = k1[i];
      c.sm[L < kKA ? SB::K2 + t * kKA + L : SB::SPARE] = ka[i];
      c.sm[L < kKA && 16 + t < kL2 ? SB::K2 + (16 + t) * kKA + L : SB::SPARE] = kb[i];
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = 4 * q + i;
    c.sm[L < kKA ? SM_K1 + t * kKP + L : SB::SPARE] = k1[i];
    c.sm[L < kKA ? SB::K2 + (t < kL ? t : t + 4) * kKP + L : SB::SPARE] = ka[i];
    c.sm[L < kKA && 16 + t < kL2 ? SB::K2 + (20 + t) * kKP + L : SB::SPARE] = kb[i];
  }
}

// PAD: the frame heads' zero-padded operands that are not K1 / K2 values, in
// one wave of the first staging (a task of its own: beside K1 / K2, not
// after them) — K2's zero rows 12..15 and 28..31, the scene's lambda G
// ([16][16], columns 8..15 zero), the augmented operands' constant rows: V
// row wcmax + 2 = bv, V and VG rows wcmax + 3 = 0 (no chunk's staging writes
// those rows, so once per scene).
__device__ __forceinline__ void scene_pad_consts(const SceneCtx& c, const SceneLayout& lay,
                                                 float lambda) {
  using SB = SmallBlock<true>;
  const int L = c.L, q = c.q;
  const float* sm = c.sm;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = c.lane + 64 * j, r = idx / kKA;
    if (idx < 8 * kKA) c.sm[SB::K2 + (r < 4 ? kL + r : 24 + r) * kKP + idx % kKA] = 0.f;
  }
  // lambda G: lane (L, q) writes row L, columns 4q .. 4q + 3 (zero for q >= 2)
  {
    const float4 g = *reinterpret_cast<const float4*>(sm + SM_G + L * kT + 4 * (q & 1));
    *reinterpret_cast<float4*>(c.sm + SB::LG + L * kGP + 4 * q) =
        q < 2 ? make_float4(lambda * g.x, lambda * g.y, lambda * g.z, lambda * g.w)
              : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (q < 3) {
    float* dst = q == 0 ? c.sV + (lay.wcmax + 2) * kD : q == 1 ? c.sV + (lay.wcmax + 3) * kD
                                                                : c.sVG + (lay.wcmax + 3) * kD;
    dst[L] = q == 0 ? sm[SM_BV + L] : 0.f;
  }
}

// NLL loss: the head's per-step constants from its raw values (one lane per
// step): 1/sigma_x, 1/sigma_y, rho, 1/(1 - rho^2), log(2 pi) + log sigma_x +
// log sigma_y + 1/2 log(1 - rho^2), as g2k_nll_kernel forms them.
__device__ __forceinline__ void scene_nll_consts(const SceneCtx& c) {
  const int t = c.lane;
  if (t < kL) {
    const float lsx = c.sNllR[t], lsy = c.sNllR[kL + t], r = c.sNllR[2 * kL + t];
    const float rho = tanhf(r), cc = 1.f - rho * rho;
    c.sNllC[t] = expf(-lsx);
    c.sNllC[kL + t] = expf(-lsy);
    c.sNllC[2 * kL + t] = rho;
    c.sNllC[3 * kL + t] = 1.f / cc;
    c.sNllC[4 * kL + t] = 1.8378770664093453f + lsx + lsy + 0.5f * logf(cc);
  }
}

// Rm = Wr @ Rel, Rel = Ve * Ve (train.py:194-195, g2k_lstm_mcr.py:106):
// rows t = 4q + i of column L, zero for t >= 8 (unconditional loads, rows t
// of lane groups 2, 3 clamped, then selects)
__device__ __forceinline__ void scene_rm(const SceneLayout& lay, const SceneCtx& c, float (&rm)[4]) {
  const int L = c.L, q = c.q;
  const float ve0 = c.sV[lay.wcmax * kD + L], ve1 = c.sV[(lay.wcmax + 1) * kD + L];
  float2 wr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) wr[i] = *reinterpret_cast<const float2*>(c.sm + SM_WR + 2 * (4 * (q & 1) + i));
#pragma unroll
  for (int i = 0; i < 4; ++i)
    rm[i] = lane_sel(q < 2, fmaf(wr[i].x, ve0 * ve0, wr[i].y * (ve1 * ve1)), 0.f);
}

// Frames 0 .. n-1 whose As the recurrence waves form themselves (one frame
// per wave — two in the co-resident geometry (CR) when a frame has 3 or more
// prediction tiles, round 4: kfold4 10.8 -> 10.6 us per step, relational
// 18.7 -> 18.4, the 2-tile shapes neutral — right after the first staging;
// the scene's recurrence workgroup)
template <bool CR, bool INV>
__device__ __forceinline__ int rec_head_frames(const SceneLayout& lay, const SceneCtx& c) {
  const int n = c.nf < lay.fc ? c.nf : lay.fc;
  if (INV) return n < 1 ? n : 1;              // loop-invariant frames: frame 0's head only
  const int m = kRecW * (CR && c.ntact >= 3 ? 2 : 1);
  return n < m ? n : m;
}

// Chunk staging shared by both roles (every wave takes part).  The chunk's
// position window is in flight by LDS-DMA.  Wait, barrier; the producer
// waves compute the embedding-row tiles (scene_vtile) and, at the first
// chunk, K1 / K2 (scene_kmats) while `rec_init` runs on the recurrence
// waves; barrier.  Both barriers are raw s_barriers after the waits they
// need (__syncthreads() would also drain every load in flight).  The DMA
// wait is the s_waitcnt BUILTIN, not inline asm: the compiler's wait
// insertion then knows the LDS-DMA has landed.  (It cannot see a wait in
// inline asm; believing the DMA of a later chunk still in flight, it put a
// vmcnt(0) before the first LDS read after the staging — which drained the
// first tiles' target loads, issued to fly under the frame heads, and held
// the first head back by a full HBM round trip.)
template <int NT, int NP, bool PAD, bool NLL = false, typename RecInit>
__device__ __forceinline__ void scene_stage(const StepArgs& a, const SceneLayout& lay,
                                            const SceneCtx& c, int fb, int cnt, RecInit rec_init) {
  const int wcc = (cnt - 1) * a.d.stride + kT;
  __builtin_amdgcn_s_waitcnt(0x0070);                           // vmcnt(0) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();                                 // B1: window + weights landed
  if (c.wv >= kRecW) {
    const int ntile = (wcc + 3 + 15) / 16;
    const int ntask = ntile + (fb == 0 ? (PAD ? 2 : 1) : 0);
    auto run = [&](int task) {
      if (task < ntile) {
        scene_vtile<PAD>(a, lay, c, 16 * task, wcc);
      } else if (!PAD || task == ntile) {
        scene_kmats<PAD>(c);
        if (NLL) scene_nll_consts(c);
      } else {
        if constexpr (PAD) scene_pad_consts(c, lay, a.lambda);
      }
    };
    // forward (PAD): the first task outside the loop — a loop's preheader
    // would form every task kind's addresses (and reload spilled scalars)
    // after B1, ahead of the first task, on the lead's critical path
    int task = c.wv - kRecW;
    if (PAD && task < ntask) {
      run(task);
      task += NP;
    }
#pragma unroll 1
    for (; task < ntask; task += NP) run(task);
  } else {
    rec_init();
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);                           // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();                                 // B2: V, VG, K1, K2
}

// Role 1: the recurrence (waves 0..3).  Without h_in (gradient only, or a
// split scene's other workgroups) the waves only take part in the chunk
// barriers.  h is loaded during the first staging (after B1: the prologue's
// HBM burst, which every wave's B1 waits for, stays free of it) and its
// softmax numerators are formed there too; after B2 the waves form As of the
// first frames themselves and start the chain.
template <int TPW, int NP, bool CR, bool PAD, bool INV, bool BLK = false>
__device__ __forceinline__ void scene_recurrence(const StepArgs& a, const SceneLayout& lay,
                                                 const SceneCtx& c) {
  constexpr int NT = 64 * (kRecW + NP);
  constexpr int kRB = 16 * kRecW;
  const int H = a.d.H;
  const bool live = a.h_in != nullptr && c.x == 0;   // (the scene's first workgroup)
  RecurH<TPW, kRecW> rc;
  int* seq = reinterpret_cast<int*>(c.sRed + 2 * kRB);   // 2 partial buffers, seq words, row max
  // the first chunk's staging ahead of the chunk loop (see scene_producer);
  // the recurrence waves load h and form its softmax numerators meanwhile
  // (row max exchange: seq 1; e and its row partials into buffer 0: seq 2),
  // off the chain's critical path, which starts with the first heads after
  // the staging
  if (live && c.nf > 0) rc.load(a.h_in + (size_t)c.s * kD * H, H, c.wv, c.q, c.L);   // (in the prologue's burst)
  if (c.nf > 0)
    scene_stage<NT, NP, PAD>(a, lay, c, 0, c.nf < lay.fc ? c.nf : lay.fc, [&] {
      if (!live) return;
      rc.init_max(c.sRed + 3 * kRB, c.wv, c.q, c.L);
      asm volatile("" ::: "memory");
      if (c.lane == 0) lds_store_flag(seq + c.wv, 1);
      poll_seq(seq + (c.L & 3), 1);
      rc.init_exp(c.sRed, c.sRed + 3 * kRB, c.wv, c.q, c.L);
      asm volatile("" ::: "memory");
      if (c.lane == 0) lds_store_flag(seq + c.wv, 2);
    });
  // the first frames' attention weights (E -> A -> As into the ring, the
  // flag) by the recurrence waves themselves, one frame per wave at top
  // priority: the producers reach their first heads only after their loop
  // set-up (thousands of cycles of scalar work on the CU's one scalar unit);
  // they form only M for these frames
  for (int fl = c.wv; live && fl < rec_head_frames<CR, INV>(lay, c); fl += kRecW) {
    __builtin_amdgcn_s_setprio(3);
    float rm[4];
    scene_rm(lay, c, rm);
    const bool mine = c.X == 1 || (BLK ? frame_owner(0, c.nf < lay.fc ? c.nf : lay.fc, fl, c.X, lay.own0) : fl % c.X) == 0;
    // the co-resident geometry: these frames' M too (its producers skip
    // them).  Not in train mode: there the producers form these frames' M
    // AND the cost their gradient terms read (sCost), and the M flag must not
    // be published before that cost is in LDS
    constexpr bool kRecM = CR;
    const FrameHeadOut hd =
        frame_head<PAD, INV>(c.sm, c.sV, c.sVG, fl * a.d.stride, lay.wcmax, rm, a.lambda, c.sRing + fl * kD * kD,
                   c.sFlag + fl, fl + 1,
                   a.A_out && mine ? a.A_out + ((size_t)c.s * a.d.F + fl) * kD * kD : nullptr,
                   kRecM && a.cost_out && mine ? a.cost_out + ((size_t)c.s * a.d.F + fl) * kT * kT : nullptr,
                   nullptr, c.L, c.q, /*want_m=*/kRecM && mine, true,
                   INV ? (c.nf < lay.fc ? c.nf : lay.fc) : 1);
    if (kRecM && mine) {
      if (c.L < kL && c.q < 2) {
        float* m = c.sMring + fl * kL2 * kT;
        *reinterpret_cast<float4*>(m + c.L * kT + 4 * c.q) = make_float4(hd.mT0[0], hd.mT0[1], hd.mT0[2], hd.mT0[3]);
        *reinterpret_cast<float4*>(m + (kL + c.L) * kT + 4 * c.q) = make_float4(hd.mT1[0], hd.mT1[1], hd.mT1[2], hd.mT1[3]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (c.lane == 0) lds_store_flag(c.sMflag + fl, fl + 1);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  for (int fb = 0; fb < c.nf; fb += lay.fc) {
    const int cnt = (c.nf - fb) < lay.fc ? (c.nf - fb) : lay.fc;
    if (fb > 0) {
      scene_pos_dma<NT>(a, lay, c, fb, cnt);
      scene_stage<NT, NP, PAD>(a, lay, c, fb, cnt, [] {});
    }
    if (INV && live) {
      // loop-invariant frames: the chunk's one As (its local frame 0's slot,
      // flagged fb + 1) for every frame; the chain itself is unchanged
      __builtin_amdgcn_s_setprio(2);
      const float* as_lane = c.sRing + c.L * kD + 4 * c.q;
      float4 b;
      wait_as(c.sFlag, fb + 1, as_lane, b);
      for (int fl = 0; fl < cnt; ++fl) {
        const int g = fb + fl;
        f32x4 z;
        poll_red(seq + (c.L & 3), g + 2, c.sRed + (g & 1) * kRB + (c.L & 3) * 16 + 4 * c.q, z);
        int fln;
        float4 bn;
        rc.step_seq(b, z, c.sRed + ((g + 1) & 1) * kRB, seq, g + 3, c.wv, c.q, c.L, c.sFlag, as_lane,
                    fln, bn, g + 1 == c.nf);
      }
      __builtin_amdgcn_s_setprio(0);
    } else if (live) {
      __builtin_amdgcn_s_setprio(2);
      const float* as_lane = c.sRing + c.L * kD + 4 * c.q;   // this lane's As row quad, ring slot 0
      // one frame; (b, flq): this frame's prefetched As quad and flag, (bn,
      // fln): where the next frame's prefetch goes.  Unrolled by two with the
      // pairs swapped so that a prefetch never needs a register copy (a copy
      // at the loop edge waits for every outstanding LDS op, the publish too).
      auto frame = [&](int fl, float4& b, int& flq, float4& bn, int& fln) {
        const int g = fb + fl;                 // global frame index
        f32x4 z;
        poll_red(seq + (c.L & 3), g + 2, c.sRed + (g & 1) * kRB + (c.L & 3) * 16 + 4 * c.q, z);
        if (__builtin_amdgcn_readfirstlane(flq) != g + 1)
          wait_as(c.sFlag + fl, g + 1, as_lane + fl * kD * kD, b);
        const int fn = fl + 1 < cnt ? fl + 1 : fl;   // next frame's ring slot (itself at the end)
        rc.step_seq(b, z, c.sRed + ((g + 1) & 1) * kRB, seq, g + 3, c.wv, c.q, c.L, c.sFlag + fn,
                    as_lane + fn * kD * kD, fln, bn, g + 1 == c.nf);
      };
      float4 b0, b1;
      int f0 = read_as(c.sFlag, as_lane, b0), f1 = 0;
      for (int fl = 0; fl < cnt; fl += 2) {
        frame(fl, b0, f0, b1, f1);
        if (fl + 1 < cnt) frame(fl + 1, b1, f1, b0, f0);
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (fb + lay.fc < c.nf) __syncthreads();                    // B3: chunk done (not after the last)
  }
  if (!live) return;
  if (c.nf == 0) rc.load(a.h_in + (size_t)c.s * kD * H, H, c.wv, c.q, c.L);   // h passes unchanged
  // epilogue straight off the last frame: wait for every wave's last
  // partials (its sequence word), h = adj * h', store; no workgroup barrier
  // (the producers finish the metrics on their own, scene_producer)
  if (c.nf > 0) poll_seq_all(seq, c.nf + 2);
  rc.store(a.h_out + (size_t)c.s * kD * H, H, c.wv, c.q, c.L,
           c.nf > 0 ? c.sRed + (c.nf & 1) * kRB : nullptr);
}

// LDS hand-off between the lanes of ONE wave: DS instructions of a wave
// complete in issue order, so only compiler reordering has to be fenced
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One 16-pedestrian tile of one frame (models/g2k_lstm_mcr.py:122-124):
// Y = M @ Wo with M = this frame's [24][8] from the M ring.  The rows are
// taken in the targets' interleaved order r = 2 step + xy (physical M / pred
// row mrow(r)), so lane (L, q) ends with Y[r][n0 + L] for r = 4q + v (block
// 0) and r = 16 + 4q + v (block 1, q < 2): pedestrian n0 + L, steps 2q, 2q+1
// and 8+2q, 9+2q, exactly the two float4s of its target row it loaded (tg).
// The a9 error terms (train.py:640-656) are per-lane sums over those steps,
// then across the four lane groups (permlane swaps); no LDS transpose.
// pred stores: active columns only (n < n_active), one 64-B row segment per
// lane group and row.
// GRAD: dY = (Y - target) on active, masked pedestrians, its squares into
// lsum, and the tile's products:
//   dWoT  = dY^T @ M     (from the registers; lane (L, q) reg v: dWo[t = L][n0 + 4q + v])
//   dm   += dY @ Wo^T    (dY through the wave's [24][17] scratch; dm[0][v] =
//                         dM[r = 4q + v][t = L], dm[1][v] = dM[r = 16 + 4q + v][t = L],
//                         accumulated over the frame's tiles in registers)
__device__ __forceinline__ int mrow(int r) { return (r & 1) * kL + (r >> 1); }

// `after_targets` runs once the target registers are consumed (GRAD: the
// next tile's targets are loaded into them there, before this tile's stores,
// so the next tile's wait counts exactly those stores).
// NLL (train mode): the loss of this lane's four (x, y) pairs — steps 2q, 2q+1
// (d0) and 8+2q, 9+2q (d1, q < 2) — around pred with the head's per-step
// constants (sC [5][12]); d0 / d1 (= Y - target) are replaced by d nll / d Y,
// the nll is added to lsum and the head's gradient terms (d/dlog sigma_x,
// d/dlog sigma_y, d/datanh rho of pair j) into the lane's LDS sums sA[(3 j + k)
// * 64] (lane-minor: conflict-free).  One pair at a time, its constants and
// sums loaded right before use (few live registers: the caller is at the
// VGPR limit).
__device__ __forceinline__ void nll_pairs(const float* sC, float* sA, int q, bool has_t,
                                          float (&d0)[4], float (&d1)[4], float& lsum) {
  const bool hi = q < 2;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    asm volatile("" ::: "memory");                           // keep each pair's loads here
    const bool blk1 = j >= 2;
    const int st = blk1 ? (hi ? 8 + 2 * q + (j & 1) : 8) : 2 * q + (j & 1);
    const float w = (has_t && (!blk1 || hi)) ? 1.f : 0.f;
    float* d = blk1 ? d1 : d0;
    const float isx = sC[st], isy = sC[kL + st], rho = sC[2 * kL + st], ic = sC[3 * kL + st],
                base = sC[4 * kL + st];
    float* g = sA + 3 * j * 64;
    const float g0 = g[0], g1 = g[64], g2 = g[128];
    const float a = -d[2 * (j & 1)] * isx, b = -d[2 * (j & 1) + 1] * isy;   // (target - mu) / sigma
    const float ab = a * b, z = fmaf(a, a, fmaf(b, b, -2.f * rho * ab));
    lsum = fmaf(w, fmaf(0.5f * ic, z, base), lsum);
    d[2 * (j & 1)] = w * (-(a - rho * b) * ic * isx);
    d[2 * (j & 1) + 1] = w * (-(b - rho * a) * ic * isy);
    g[0] = fmaf(w, 1.f - (a * a - rho * ab) * ic, g0);
    g[64] = fmaf(w, 1.f - (b * b - rho * ab) * ic, g1);
    g[128] = fmaf(w, -rho - ab + rho * z * ic, g2);
  }
}

// REP (forward, frames_invariant): the tile stands for `nrep` frames with the
// same values — its stores are repeated at `pr`'s consecutive frames and its
// a9 terms enter the sums with weight nrep (the count with nrep pairs).
template <bool GRAD, bool PM, bool NLL, bool REP = false, typename AfterTargets>
__device__ __forceinline__ void pred_tile(const float* M, const float* sWo, float* ys, brsrc pr,
                                          const float2 (&tg)[4], bool has_t, int Nmax, int nact,
                                          int t, int L, int q, float acc[5], float& lsum,
                                          f32x4 (&dm)[2], f32x4& dWoT, AfterTargets after_targets,
                                          const float* nllC = nullptr, float* nllA = nullptr,
                                          int nrep = 1) {
  if (GRAD && NLL) asm volatile("" : "+v"(L), "+v"(q));   // (as in frame_grad<OPAQUE>)
  const int n0 = 16 * t, n = n0 + L;
  const bool hi = q < 2;                                   // block-1 rows exist (r < 24)
  f32x4 y0 = {0.f, 0.f, 0.f, 0.f}, y1 = {0.f, 0.f, 0.f, 0.f};
  float bm[8];                                             // GRAD: M[r][t = L & 7], r as in dWoT
  {
    // unconditional loads at clamped addresses, selects after (see frame_head)
    const int nc = n < Nmax ? n : Nmax - 1, L7 = L & 7;
    float a0[2], a1[2], wo[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int k = 4 * ks + q;
      a0[ks] = M[mrow(L) * kT + k];                        // A[r = L][k]
      a1[ks] = M[mrow(16 + L7) * kT + k];                  // A[r = 16 + L][k]
      wo[ks] = sWo[k * Nmax + nc];                         // B[k][n = n0 + L]
    }
    asm volatile("" : "+v"(a0[0]), "+v"(a0[1]), "+v"(a1[0]), "+v"(a1[1]), "+v"(wo[0]), "+v"(wo[1]));
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const float w = n < nact ? wo[ks] : 0.f;
      y0 = mfma4(a0[ks], w, y0);                           // Y[4q + v][n]
      y1 = mfma4(L < kT ? a1[ks] : 0.f, w, y1);            // Y[16 + 4q + v][n] (0 for q >= 2)
    }
  }
  // errors: d = Y - target, (x, y) pairs in registers (v = 0, 1 and 2, 3)
  float d0[4], d1[4];
#pragma unroll
  for (int v = 0; v < 2; ++v) {
    d0[2 * v] = y0[2 * v] - tg[v].x;       d0[2 * v + 1] = y0[2 * v + 1] - tg[v].y;
    d1[2 * v] = hi ? y1[2 * v] - tg[2 + v].x : 0.f;
    d1[2 * v + 1] = hi ? y1[2 * v + 1] - tg[2 + v].y : 0.f;
  }
  after_targets();
  asm volatile("" ::: "memory");                           // ... then the stores
  if (PM) {
    // pedestrian-major [Nmax][L][2]: the lane's Y values ARE its target row's
    // floats 4q..4q+3 and 16+4q..16+4q+3 (r = 2 step + xy), so two 16-byte
    // stores at the offsets of its two target loads; pedestrians >= n_active
    // are not written (a contiguous n_active * 96-byte run per frame)
    const int off = n * kL2 * 4;
    if constexpr (REP) {
      for (int r = 0; r < nrep; ++r) {
        const int fo = r * (kL2 * Nmax * 4);
        bstore4(pr, n < nact ? fo + off + 16 * q : kBufOff, y0[0], y0[1], y0[2], y0[3]);
        bstore4(pr, (n < nact && hi) ? fo + off + 64 + 16 * q : kBufOff, y1[0], y1[1], y1[2], y1[3]);
      }
    } else {
      bstore4(pr, n < nact ? off + 16 * q : kBufOff, y0[0], y0[1], y0[2], y0[3]);
      bstore4(pr, (n < nact && hi) ? off + 64 + 16 * q : kBufOff, y1[0], y1[1], y1[2], y1[3]);
    }
  } else if constexpr (REP) {
    for (int r = 0; r < nrep; ++r) {
      const int fo = r * (kL2 * Nmax * 4);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        bstore(pr, n < Nmax ? fo + (mrow(4 * q + v) * Nmax + n) * 4 : kBufOff, y0[v]);
        bstore(pr, (n < Nmax && hi) ? fo + (mrow(16 + 4 * q + v) * Nmax + n) * 4 : kBufOff, y1[v]);
      }
    }
  } else {
    // range-checked 4-byte stores (no branch): the block-1 rows of lane
    // groups 2, 3 and columns past Nmax fall outside the frame's buffer.  The
    // tile's 16 columns are written whole (Y = 0 past n_active, w = 0 there):
    // 64-byte row segments, where a partial one costs the memory side a
    // read-modify-write once the output is not cache-resident (rotated
    // outputs: 21.5 -> 20.7 us per step at eth_hotel_synth)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      bstore(pr, n < Nmax ? (mrow(4 * q + v) * Nmax + n) * 4 : kBufOff, y0[v]);
      bstore(pr, (n < Nmax && hi) ? (mrow(16 + 4 * q + v) * Nmax + n) * 4 : kBufOff, y1[v]);
    }
  }
  if (GRAD && !NLL) {
    // M's operand of dWo^T, loaded here (not with Y's operands) so that it is
    // not live across the stores; its latency hides under the error terms
    // (NLL: after the loss terms, which need the registers first)
    const int L7 = L & 7;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bm[ks] = M[mrow(4 * q + ks) * kT + L7];
      bm[4 + ks] = M[mrow(16 + 4 * (q & 1) + ks) * kT + L7];
    }
    asm volatile("" : "+v"(bm[0]), "+v"(bm[1]), "+v"(bm[2]), "+v"(bm[3]), "+v"(bm[4]), "+v"(bm[5]),
                 "+v"(bm[6]), "+v"(bm[7]));
  }
  float ea = 0.f, eb = 0.f, ec = 0.f, el2 = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float* d = h ? d1 : d0;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const float dx = d[2 * v], dy = d[2 * v + 1];
      ea = fmaf(dx, dx, ea);
      eb = fmaf(dx, dy, eb);
      ec = fmaf(dy, dy, ec);
      el2 += __builtin_amdgcn_sqrtf(fmaf(dx, dx, dy * dy));
    }
  }
  // el2 needs no sum across lanes: each lane adds its steps' share (the
  // lanes are summed when the metrics are published)
  const float wrep = REP ? (float)nrep : 1.f;
  acc[3] = fmaf(has_t ? wrep * (1.0f / 12.0f) : 0.f, el2, acc[3]);
  // ea, eb, ec summed over the four lane groups and gathered in group 1 (it
  // holds step 11, the fde) by five permlane swaps, branch-free after.
  // permlane32_swap(x, y) -> {[x.lo, y.lo], [x.hi, y.hi]} (32-lane halves);
  // permlane16_swap(x, y) -> {[x.r0, y.r0, x.r2, y.r2], [x.r1, y.r1, x.r3, y.r3]}
  auto sw32 = [](float x, float y) {
    return __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  };
  auto sw16 = [](float x, float y) {
    return __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  };
  const auto p1 = sw32(ea, eb), p2 = sw32(ec, ec);
  const float s1 = __uint_as_float(p1[0]) + __uint_as_float(p1[1]);   // rows: ea, ea, eb, eb (halves)
  const float s2 = __uint_as_float(p2[0]) + __uint_as_float(p2[1]);   // ec halves
  const auto p3 = sw16(s1, s2);
  const float tt = __uint_as_float(p3[0]) + __uint_as_float(p3[1]);   // rows: ea, ec, eb, ec
  const auto p4 = sw16(tt, tt);                                       // [0]: rows ea, ea, eb, eb
  const auto p5 = sw32(__uint_as_float(p4[0]), __uint_as_float(p4[0]));   // [1]: eb everywhere
  const float sa = __uint_as_float(p4[0]), sb = __uint_as_float(p5[1]), sc = tt;   // row 1
  {
    const float g1 = (has_t && q == 1) ? wrep : 0.f;   // group 1's lanes of pedestrians with targets
    const float fx = d1[2], fy = d1[3];
    const float hm = 0.5f * (sa - sc);
    const float lam = 0.5f * (sa + sc) + __builtin_amdgcn_sqrtf(fmaf(hm, hm, sb * sb));
    const float fsq = fmaf(fx, fx, fy * fy);
    acc[0] = fmaf(g1 * (1.0f / 12.0f), __builtin_amdgcn_sqrtf(fmaxf(lam, 0.f)), acc[0]);
    acc[1] += g1;
    acc[2] = fmaf(g1, fsq, acc[2]);
    acc[4] = fmaf(g1, __builtin_amdgcn_sqrtf(fsq), acc[4]);
    if (GRAD && !NLL) lsum = fmaf(g1, sa + sc, lsum);
  }
  if (GRAD) {
    if (NLL) {
      nll_pairs(nllC, nllA, q, has_t, d0, d1, lsum);         // dY = d nll / d Y (masked)
      const int L7 = L & 7;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        bm[ks] = M[mrow(4 * q + ks) * kT + L7];
        bm[4 + ks] = M[mrow(16 + 4 * (q & 1) + ks) * kT + L7];
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      d0[v] = has_t ? d0[v] : 0.f;
      d1[v] = has_t ? d1[v] : 0.f;
    }
    // dY into the scratch [r][n] (pitch kYP) for dM, where n must be the
    // contraction index
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      ys[(4 * q + v) * kYP + L] = d0[v];
      if (hi) ys[(16 + 4 * q + v) * kYP + L] = d1[v];
    }
    // dWo^T = dY^T @ M: A[n = L][r] = dY[r][n0 + L] (registers), B[r][t = L] = M[r][t]
    {
      f32x4 w = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) w = mfma4(d0[ks], bm[ks], w);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) w = mfma4(d1[ks], hi ? bm[4 + ks] : 0.f, w);
      dWoT = w;
    }
    wave_lds_sync();
    // dm += dY @ Wo^T: A[r = L][n] = dY[r][n0 + n] (scratch), B[n][t = L] = Wo[t][n0 + n]
    {
      float a0[4], a1[4], bw[4];
      const int L7 = L & 7;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int k = 4 * ks + q, nk = n0 + k;
        a0[ks] = ys[L * kYP + k];
        a1[ks] = ys[(16 + L7) * kYP + k];
        bw[ks] = sWo[L7 * Nmax + (nk < Nmax ? nk : Nmax - 1)];
      }
      asm volatile("" : "+v"(a0[0]), "+v"(a0[1]), "+v"(a0[2]), "+v"(a0[3]), "+v"(a1[0]), "+v"(a1[1]),
                   "+v"(a1[2]), "+v"(a1[3]), "+v"(bw[0]), "+v"(bw[1]), "+v"(bw[2]), "+v"(bw[3]));
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        dm[0] = mfma4(a0[ks], bw[ks], dm[0]);
        dm[1] = mfma4(L < kT ? a1[ks] : 0.f, bw[ks], dm[1]);
      }
    }
    wave_lds_sync();                       // scratch reads done before the next tile's writes
  }
}

// Wait (one LDS word, wave-uniform) until *w == want.
__device__ __forceinline__ void poll_word(const int* w, int want) { poll_flag(w, want); }

// D = A @ B on one 16 x 16 tile by v_mfma_f32_16x16x4_f32 with k = 4 ks + q:
// lane (L, q) supplies A(L, k) and B(k, L) at k-step ks (the functors load
// unconditionally at clamped LDS addresses and select), every load issued
// before the first MFMA; the result lands as D(4q + v, L) in register v.
template <int KS, typename FA, typename FB>
__device__ __forceinline__ f32x4 mm16(FA fa, FB fb, int L, int q) {
  float av[KS], bv[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    av[ks] = fa(L, 4 * ks + q);
    bv[ks] = fb(4 * ks + q, L);
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) acc = mfma4(av[ks], bv[ks], acc);
  return acc;
}

// GRAD, after the last tile of chunk frame fl: the frame's weight-side
// terms (one wave, MFMA tiles from LDS) added into this producer's own sums
// (sGPriv: dWc, dK1, dVe, dbv; sGPdV: the chunk's window rows) — each entry
// by one lane of one wave, in the producer's frame order: deterministic
// without any cross-wave ordering; grad_chunk_flush / grad_priv_sum add the
// producers' sums in producer order.
//   dcost[u][t] = sum_r Wc[r][u] dM[r][t]          (M = Wc @ cost, :119)
//   dE[t][d]    = lambda sum_u dcost[t][u] G[d][u] (cost = E @ g, :112-113)
//   dWc_f[r][u] = sum_t dM[r][t] cost[u][t]
//   dK1_f[t][j] = sum_d dE[t][d] Uaug[j][d]        (E = K1 @ Uaug, j < 10)
//   dUaug_f[j][d] = sum_t K1[t][j] dE[t][d]        (j < 8: window rows, 8-9: Ve, 10: bv)
// REP (frames_invariant): the frame stands for `wrep` frames with the same
// terms; they enter the sums with that weight.
template <bool OPAQUE, bool REP = false>
__device__ __forceinline__ void frame_grad(const StepArgs& a, const SceneLayout& lay,
                                           const SceneCtx& c, int fl, const f32x4 (&dm)[2],
                                           int slot, float wrep = 1.f) {
  // The products chain through the MFMA registers: a result D (lane (L, q)
  // reg v = D[4q+v][L]) is the next product's B operand as is (k = 4q + ks
  // <-> reg ks) or its A operand transposed (A[L][4q+ks] = D[4q+ks][L]), so
  // only the constant operands and dWc's dM come from LDS.
  //   P1 dcost^T[t2][t1] = sum_r dM[r][t2] Wc[r][t1]      (A: dm registers,
  //                                                         rows r interleaved)
  //   P2 dE[t1][d]   = lambda sum_t2 dcost[t1][t2] G[d][t2]   (A: P1^T)
  //   P3 dE^T[d][t1] = lambda sum_t2 G[d][t2] dcost^T[t2][t1] (B: P1)
  //   P4 dU[j][d]    = sum_t1 K1[t1][j] dE[t1][d]          (B: P2)
  //   P5 dK1[t1][j]  = sum_d dE[t1][d] Uaug[j][d]          (A: P3^T)
  //   P6 dWc[r][t1]  = sum_t2 dM[r][t2] cost[t1][t2]       (dM from LDS)
  const float* dM = c.sGFrame + slot * kGFrame + kGT_DM;
  float* pacc = c.sGPriv + slot * kGAccFixed;
  float* pdv = c.sGPdV + slot * lay.wcmax * kD + fl * a.d.stride * kD;
  // OPAQUE (the NLL builds): the lane indices made opaque per call, so its
  // LDS addresses are formed here, not hoisted into the producer's preheader
  // and held across the whole role — the NLL kernels' register peak
  // (spill-free then: eth_hotel_synth NLL train 56.3 -> 52.6 us per step;
  // the L2 builds, with registers to spare, lose 3 us to the re-formed
  // addresses: DESIGN.md §11)
  int L = c.L, q = c.q;
  if (OPAQUE) asm volatile("" : "+v"(L), "+v"(q));
  const int L7 = L & 7, q1 = q & 1;
  const float* sm = c.sm;
  const float* cost = c.sCost + fl * kT * kT;
  const int wrow0 = fl * a.d.stride;
  const int jr = L < kT ? wrow0 + L : lay.wcmax + (L < kT + 2 ? L - kT : 1);   // Uaug row j = L
  // every operand load first (clamped addresses), selects after
  float wc[8], gq[4], k1[4], ua[4], mA[4], cB[2];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    // dm's rows r are in the tiles' interleaved order: Wc row mrow(r)
    wc[ks] = sm[SM_WC + mrow(4 * q + ks) * kT + L7];              // Wc[r = 4q+ks][t1 = L]
    wc[4 + ks] = sm[SM_WC + mrow(16 + 4 * q1 + ks) * kT + L7];    // Wc[16 + 4q+ks][t1]
    gq[ks] = sm[SM_G + L * kT + 4 * q1 + ks];                     // G[d = L][t2 = 4q+ks]
    k1[ks] = sm[SM_K1 + (4 * q1 + ks) * kKA + (L < kKA ? L : 0)]; // K1[t1 = 4q+ks][j = L]
    ua[ks] = c.sV[jr * kD + 4 * q + ks];                          // Uaug[j = L][d = 4q+ks]
  }
  wave_lds_sync();                                        // the frame's dM in LDS (P6)
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const int t2 = 4 * ks + q;
    mA[2 * ks] = dM[L * kT + (t2 & 7)];                           // dM[r = L][t2]
    mA[2 * ks + 1] = dM[(16 + L7) * kT + (t2 & 7)];               // dM[16 + L][t2]
    cB[ks] = cost[L7 * kT + (t2 & 7)];                            // cost[t1 = L][t2]
  }
  asm volatile("" : "+v"(wc[0]), "+v"(wc[1]), "+v"(wc[2]), "+v"(wc[3]), "+v"(wc[4]), "+v"(wc[5]),
               "+v"(wc[6]), "+v"(wc[7]), "+v"(gq[0]), "+v"(gq[1]), "+v"(gq[2]), "+v"(gq[3]));
  asm volatile("" : "+v"(k1[0]), "+v"(k1[1]), "+v"(k1[2]), "+v"(k1[3]), "+v"(ua[0]), "+v"(ua[1]),
               "+v"(ua[2]), "+v"(ua[3]), "+v"(mA[0]), "+v"(mA[1]), "+v"(mA[2]), "+v"(mA[3]),
               "+v"(cB[0]), "+v"(cB[1]));
  const bool lo = q < 2;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    wc[4 + ks] = lo ? wc[4 + ks] : 0.f;                           // rows r >= 24
    gq[ks] = lo ? a.lambda * gq[ks] : 0.f;                        // t2 >= 8
    k1[ks] = (lo && L < kT + 3) ? k1[ks] : 0.f;                   // t1 >= 8, j >= 11
    ua[ks] = L < kT + 2 ? ua[ks] : 0.f;                           // j >= 10
  }
  // P1
  f32x4 dcT = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) dcT = mfma4(dm[0][ks], wc[ks], dcT);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) dcT = mfma4(dm[1][ks], wc[4 + ks], dcT);
  // P6 (independent of P1..P5)
  f32x4 w0 = {0.f, 0.f, 0.f, 0.f}, w1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const float cb = L < kT ? cB[ks] : 0.f;
    w0 = mfma4(mA[2 * ks], cb, w0);                               // dWc[4q+v][t1 = L]
    w1 = mfma4(L < kT ? mA[2 * ks + 1] : 0.f, cb, w1);            // dWc[16 + 4q+v][t1]
  }
  // P2, P3
  f32x4 dE = {0.f, 0.f, 0.f, 0.f}, dET = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    dE = mfma4(dcT[ks], gq[ks], dE);
    dET = mfma4(gq[ks], dcT[ks], dET);
  }
  // P4, P5
  f32x4 dU = {0.f, 0.f, 0.f, 0.f}, dK = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    dU = mfma4(k1[ks], lo ? dE[ks] : 0.f, dU);
    dK = mfma4(dET[ks], ua[ks], dK);
  }
  // into this producer's sums
  if constexpr (REP) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      w0[v] *= wrep; w1[v] *= wrep; dK[v] *= wrep; dU[v] *= wrep;
    }
  }
  if (L < kT) {
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      pacc[kGA_WC + (4 * q + v) * kT + L] += w0[v];
      if (lo) pacc[kGA_WC + (16 + 4 * q + v) * kT + L] += w1[v];
    }
  }
  if (lo && L < kT + 2) {
#pragma unroll
    for (int v = 0; v < 4; ++v) pacc[kGA_K1 + (4 * q + v) * 10 + L] += dK[v];
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int j = 4 * q + v;                              // window rows, Ve0, Ve1, bv
    if (j < kT) pdv[j * kD + L] += dU[v];
    else if (j < kT + 2) pacc[kGA_VE + (j - kT) * kD + L] += dU[v];
    else if (j == kT + 2) pacc[kGA_BV + L] += dU[v];
  }
  wave_lds_sync();                                        // before the next frame's dM
}

// GRAD, once every producer is done with chunk [fb, fb + cnt): the
// producers' dU rows of the chunk added into the scene's window-row gradient
// dV in producer order (one entry per producer lane, the chunk's rows), then
// zeroed for the next chunk.
__device__ __forceinline__ void grad_chunk_flush(const StepArgs& a, const SceneLayout& lay,
                                                 const SceneCtx& c, int fb, int cnt, int NP) {
  const int NG = NP + kRecW;
  const int r0 = fb * a.d.stride, nrow = (cnt - 1) * a.d.stride + kT;
  const int ptid = (c.wv - kRecW) * 64 + c.lane;
  const int pitch = lay.wcmax * kD;
  for (int e = ptid; e < nrow * kD; e += NP * 64) {
    float v[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) v[p] = p < NG ? c.sGPdV[p * pitch + e] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (p < NG) s += v[p];                                 // worker order
    c.sGdV[r0 * kD + e] += s;
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (p < NG) c.sGPdV[p * pitch + e] = 0.f;
  }
}

// GRAD, after every producer's last frame: sGAcc = the producers' fixed-block
// sums (dWc, dK1, dVe, dbv) added in producer order.
__device__ __forceinline__ void grad_priv_sum(const SceneCtx& c, int NP) {
  const int NG = NP + kRecW;
  const int ptid = (c.wv - kRecW) * 64 + c.lane;
  for (int e = ptid; e < kGAccFixed; e += NP * 64) {
    float v[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) v[p] = p < NG ? c.sGPriv[p * kGAccFixed + e] : 0.f;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (p < NG) s += v[p];
    c.sGAcc[e] = s;
  }
}

// This lane's dword of the scene's ped_mask row (pedestrians 4 lane ..
// 4 lane + 3; all ones without a mask).  A dword-aligned row arrived with the
// prologue's LDS-DMA (segment 11): one LDS read.  (Loaded at the top of the
// producer role, it was a dependent HBM miss behind the n_active scalar
// load that every producer waited for before the staging barrier.)  Rows
// that are not dword-aligned are read from global memory here.
__device__ __forceinline__ bool mask_one_load(const StepArgs& a) {
  return a.ped_mask && (a.d.Nmax & 3) == 0 && (((uintptr_t)a.ped_mask) & 3) == 0;
}
__device__ __forceinline__ uint32_t scene_mask_word(const StepArgs& a, const SceneLayout& lay,
                                                    const SceneCtx& c) {
  const int Nmax = a.d.Nmax;
  if (!a.ped_mask) return ~0u;
  // (the lane index made opaque: the loop-invariant addresses below would be
  // formed in the prologue and held, a spill, at the register limit)
  int lane = c.lane;
  asm volatile("" : "+v"(lane));
  if (mask_one_load(a)) {   // the LDS row, addressed from the small block: no pointer of its own
    const int l = lane < Nmax / 4 ? lane : 0;
    return reinterpret_cast<const uint32_t*>(c.sm + (lay.o_mask - lay.o_small))[l];
  }
  const uint8_t* pm = a.ped_mask + (size_t)c.s * Nmax;
  uint32_t w = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) {
    const int n = 4 * lane + b;
    w |= (uint32_t)(n < Nmax ? pm[n] : 0) << (8 * b);
  }
  return w;
}

// Pedestrian n = 16 t + L has targets (n < n_active and its ped_mask byte
// set): bit t of the lane's word.  The mask row comes as one dword per lane
// (w = scene_mask_word: pedestrians 4l .. 4l + 3 in lane l) and is spread by
// four ballots: one global round trip per wave, not one per 64 pedestrians.
__device__ __forceinline__ unsigned scene_act_bits(const SceneCtx& c, uint32_t w) {
  unsigned long long B[4];   // bit l: pedestrian 4 l + b has a target
#pragma unroll
  for (int b = 0; b < 4; ++b) B[b] = __builtin_amdgcn_ballot_w64(((w >> (8 * b)) & 0xffu) != 0);
  const int b = c.L & 3;
  const unsigned long long mine = b == 0 ? B[0] : b == 1 ? B[1] : b == 2 ? B[2] : B[3];
  // bits 4 t + L / 4 of `mine` (t = 0..15) gathered into bits t: a
  // shift-and-mask compression instead of one 64-bit shift per tile
  unsigned long long x = (mine >> (c.L >> 2)) & 0x1111111111111111ull;
  x = (x | (x >> 3)) & 0x0303030303030303ull;
  x = (x | (x >> 6)) & 0x000F000F000F000Full;
  x = (x | (x >> 12)) & 0x000000FF000000FFull;
  x = (x | (x >> 24)) & 0xFFFFull;
  // and only tiles t with 16 t + L < n_active
  const int nt = c.nact > c.L ? (c.nact - c.L + 15) >> 4 : 0;
  return (unsigned)x & ((1u << nt) - 1u);
}

// Train mode: the last R frames of the scene's last chunk go to the
// recurrence waves (one each, after their recurrence), so the producers'
// share shrinks when they have at least two frames each.
__device__ __forceinline__ int grad_rec_frames(int cnt, int NP, bool live) {
  // a workgroup without the chain (a split scene's other workgroups): its
  // recurrence waves are free from the start — whole frames, one each, the
  // frames past one per producer (dense_crowd's 11 of 20: 101.2 -> 99.8 us
  // per train step, profiles/r12v_*)
  if (!live) return cnt > NP ? (cnt - NP < kRecW ? cnt - NP : kRecW) : 0;
  return cnt >= 2 * NP ? kRecW : 0;
}
// ... split by tile when a frame has two or more: the recurrence wave takes
// tiles [0, h) (it starts at the chain's end), producer w (w < R, free after
// its own frames; the last R producers measured slower) tiles [h, ntact) of
// the same frame; each adds its partial
// dM's weight-side terms (frame_grad is linear in dM) into its own sums
__device__ __forceinline__ int grad_rec_tiles(int ntact, bool live) {
  if (!live) return ntact;
  return ntact >= 2 ? (ntact + 1) / 2 : ntact;
}

// The targets of tile t of chunk frame fl in pred_tile's order (pedestrian
// 16 t + L, floats 4q .. 4q + 3 and 16 + 4q .. 16 + 4q + 3 of its row, zero
// for q >= 2) by range-checked buffer loads (no branch: !ok and inactive
// pedestrians n >= n_active read zeros without touching memory).
// tfb = SceneLayout::tfb, the bytes between two frames' targets (0: one set
// for every frame, G2K_STEP_TARGETS_SHARED) — a kernel argument, so the
// option costs the train-mode producers no register (a per-call select of
// the flag spilled one there).
__device__ __forceinline__ void load_targets(brsrc tgr, int Nmax, int nact, int fb, int fl, int t,
                                             bool ok, int L, int q, float2 (&tg)[4], int tfb) {
  const int ne = 16 * t + L;
  ok = ok && ne < nact;
  const int base = (fb + fl) * tfb + (ne < Nmax ? ne : 0) * (kL2 * 4);
  // two 16-B loads (rows are 96 B: every float4 is 16-B aligned)
  const float4 u = bload4(tgr, ok ? base + 16 * q : kBufOff);
  const float4 w = bload4(tgr, ok && q < 2 ? base + 64 + 16 * q : kBufOff);
  tg[0] = make_float2(u.x, u.y);
  tg[1] = make_float2(u.z, u.w);
  tg[2] = make_float2(w.x, w.y);
  tg[3] = make_float2(w.z, w.w);
}

__device__ __forceinline__ brsrc scene_targets_rsrc(const StepArgs& a, int s) {
  const int tf = (a.d.flags & G2K_STEP_TARGETS_SHARED) ? 1 : a.d.F;   // target frames per scene
  return make_brsrc(a.targets + (size_t)s * tf * a.d.Nmax * kL2, (uint32_t)tf * a.d.Nmax * kL2 * 4);
}

// tile_stores out-of-range stores right after the first target load of a
// tile loop: every wait on a target load in the loop then has the same number
// of younger stores before it (a tile's own) and the compiler's counts stay
// exact (vmcnt(tile_stores), not 0).
template <bool PM>
__device__ __forceinline__ void balance_stores(const StepArgs& a) {
  asm volatile("" ::: "memory");
  const brsrc none = make_brsrc(a.targets, 0u);
#pragma unroll
  for (int i = 0; i < tile_stores<PM>(); ++i) {
    if (PM) bstore4(none, kBufOff, 0.f, 0.f, 0.f, 0.f);
    else bstore(none, kBufOff, 0.f);
  }
}

// GRAD: one gradient worker's frames fl = f0, f0 + fstep, ... < fend of the
// chunk at fb (worker `slot`: producer pw = slot, recurrence wave NP + w):
// per tile the predictions, the a9 terms, dY, dWo^T (into the worker's copy,
// or in frame order when one copy is kept), dM in registers; per frame the
// weight-side terms (frame_grad) into the worker's sums.  One target buffer:
// each tile loads the next tile's targets as soon as its own are consumed,
// before its prediction stores (tg holds the first tile's targets on entry
// when `preloaded`).
// REP (frames_invariant): frame f0 stands for the `nrep` frames fb .. fb +
// nrep - 1 — its predictions are stored for each of them, its terms enter the
// sums with weight nrep.
template <bool PM, bool NLL, bool REP = false, bool BLK = false>
__device__ __forceinline__ void grad_frames(const StepArgs& a, const SceneLayout& lay,
                                            const SceneCtx& c, int slot, int fb, int f0, int fstep,
                                            int fend, unsigned act_bits, float (&acc)[5],
                                            float& lsum, float2 (&tg)[4], bool preloaded,
                                            int t0 = 0, int t1 = -1, int nrep = 1) {
  const int Nmax = a.d.Nmax, F = a.d.F, L = c.L, q = c.q;
  const int ntact = t1 < 0 ? c.ntact : t1;             // tiles [t0, ntact) of each frame
  const brsrc tgr = scene_targets_rsrc(a, c.s);
  if (!preloaded) {
    load_targets(tgr, Nmax, c.nact, fb, f0, t0, f0 < fend, L, q, tg, lay.tfb);
    balance_stores<PM>(a);
  }
  float* ys = c.sY + slot * kL2 * kYP;
  f32x4 dm[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  for (int fl = f0; fl < fend; fl += fstep) {
    const int f = fb + fl;
    // the workgroup's own frames in order (dwo_seq): modular ownership f /
    // split; BLK: the own frames of the earlier (full) chunks, then the
    // ordinal in this chunk's block
    int ford = f / lay.split;
    if (BLK) {
      const int cnt = (c.nf - fb) < lay.fc ? (c.nf - fb) : lay.fc;
      const int nfull = own_block0(lay.fc, lay.own0), n0 = own_block0(cnt, lay.own0);
      ford = (fb / lay.fc) * (c.x == 0 ? nfull : lay.fc - nfull) + (c.x == 0 ? fl : fl - n0);
    }
    poll_flag(c.sMflag + fl, f + 1);                     // M of this frame (a producer's head)
    const brsrc pr = REP ? make_brsrc(a.pred ? a.pred + ((size_t)c.s * F + fb) * kL2 * Nmax : a.targets,
                                      a.pred ? (uint32_t)(nrep * kL2 * Nmax * 4) : 0u)
                         : make_brsrc(a.pred ? a.pred + ((size_t)c.s * F + f) * kL2 * Nmax : a.targets,
                                      a.pred ? (uint32_t)kL2 * Nmax * 4 : 0u);
    for (int t = t0; t < ntact; ++t) {
      const bool nxt = t + 1 < ntact;                    // the next tile: this frame's, else the next frame's
      const int nfl = nxt ? fl : fl + fstep, nt = nxt ? t + 1 : t0;
      f32x4 dWoT;
      pred_tile<true, PM, NLL, REP>(c.sMring + fl * kL2 * kT, c.sWo, ys, pr, tg, (act_bits >> t) & 1u,
                                    Nmax, c.nact, t, L, q, acc, lsum, dm, dWoT,
                                    [&] { load_targets(tgr, Nmax, c.nact, fb, nfl, nt, nfl < fend, L, q, tg, lay.tfb); },
                                    c.sNllC, c.sNllA + slot * 12 * 64 + c.lane, nrep);
      if constexpr (REP) {
#pragma unroll
        for (int v = 0; v < 4; ++v) dWoT[v] *= (float)nrep;
      }
      // dWo^T[n0 + 4q + v][t = L]: one copy per worker, or one copy added
      // to in frame order (tile sequence word) when that is too big
      const int nb = 16 * t + 4 * q;
      float* dst = c.sGdWo + (lay.dwo_seq ? 0 : slot * Nmax * kT);
      if (lay.dwo_seq) poll_word(c.sGseq + 2 + t, ford);
      if (L < kT) {
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (nb + v < Nmax) dst[(nb + v) * kT + L] += dWoT[v];
      }
      if (lay.dwo_seq) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (c.lane == 0) lds_store_flag(c.sGseq + 2 + t, ford + 1);
      }
    }
    // the frame's dM to this worker's scratch (M's physical rows), then its terms
    if (L < kT) {
      float* dMs = c.sGFrame + slot * kGFrame + kGT_DM;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        dMs[mrow(4 * q + v) * kT + L] = dm[0][v];
        if (q < 2) dMs[mrow(16 + 4 * q + v) * kT + L] = dm[1][v];
      }
    }
    frame_grad<NLL, REP>(a, lay, c, fl, dm, slot, (float)nrep);
    dm[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    dm[1] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

// NLL: a worker's per-lane head-gradient sums reduced over the 16 lanes
// (pedestrians) of each lane group into its row [36] (k * 12 + step): lane
// group q holds steps 2q, 2q+1 (sums 0..5) and 8+2q, 9+2q (6..11, q < 2).
__device__ __forceinline__ void nll_worker_reduce(const SceneCtx& c, int slot) {
  const float* a = c.sNllA + slot * 12 * 64 + c.lane;
  float* w = c.sNllW + slot * kNllHead;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int st = j < 2 ? 2 * c.q + j : 8 + 2 * c.q + (j - 2);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float v = row16_sum(a[(3 * j + k) * 64]);
      if (c.L == 0 && (j < 2 || c.q < 2)) w[k * kL + st] = v;
    }
  }
}

// Metrics (and the train loss): each worker publishes its partial sums in
// its row of sMet, then takes a ticket (LDS atomic); the wave drawing the
// last of `nrows` tickets sums the rows in worker order (deterministic) and
// writes the scene's metrics row.
__device__ __forceinline__ void publish_metrics(const StepArgs& a, const SceneCtx& c, int row,
                                                int nrows, const float (&acc)[5], float lsum,
                                                bool grad) {
  const int lane = c.lane;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const float v = wave_sum(acc[k]);
    if (lane == 0) c.sMet[row * 8 + k] = v;
  }
  if (grad) {
    const float v = wave_sum(lsum);
    if (lane == 0) c.sMet[row * 8 + 5] = v;
  }
  int ticket = 0;
  if (lane == 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // partials before the ticket
    ticket = atomicAdd(c.sTicket, 1);
  }
  ticket = __builtin_amdgcn_readfirstlane(ticket);
  if (ticket != nrows - 1 || !a.metrics) return;
  const int l8 = lane < 8 ? lane : 7;
  float v = 0.f;
  if (lane < 5) {
    if (c.nf > 0)
      for (int p = 0; p < nrows; ++p) v += c.sMet[p * 8 + lane];
  } else if (lane == 5) {
    v = (float)c.nf;
  }
  if (a.met_part) {
    // split scene: this workgroup's row into the scene's partials (stores that
    // write through to the coherence point, completed before the ticket); the
    // workgroup drawing the scene's last ticket sums the rows in workgroup
    // order (deterministic) after an acquire fence and writes the metrics row.
    // The tickets are zeroed in stream order before every launch
    // (scene_step_launch), so a stale or partial earlier launch cannot leave
    // one off
    const int X = c.X, x = c.x;
    float* part = a.met_part + (size_t)c.s * X * 8;
    if (lane < 8) __hip_atomic_store(part + x * 8 + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0)
      old = __hip_atomic_fetch_add(a.scene_ticket + c.s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_readfirstlane(old) != X - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (lane < 5) {
      v = 0.f;
      for (int p = 0; p < X; ++p)
        v += __hip_atomic_load(part + p * 8 + l8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (lane < 8) store_wt(a.metrics + (size_t)c.s * 8 + lane, v);
}

// Role 2: the producers (waves 4..4+NP-1).
template <int NP, bool GRAD, bool PM, bool NLL, bool CR, bool INV, bool BLK = false>
__device__ __forceinline__ void scene_producer(const StepArgs& a, const SceneLayout& lay,
                                               const SceneCtx& c) {
  const int Nmax = a.d.Nmax, F = a.d.F, stride = a.d.stride;
  const int pw = c.wv - kRecW, L = c.L, q = c.q, lane = c.lane, s = c.s, ntact = c.ntact;
  unsigned act_bits = 0;   // formed after the first staging
  // tile items of a chunk (forward): item j -> frame j / ntact, tile
  // j % ntact; this producer takes items pw, pw + NP, ...  (GRAD: whole
  // frames per worker, grad_frames)
  // item j -> (j / ntact, j % ntact) by a reciprocal, no division per item
  // (exact while j * ntact < 2^16; here j < 32 ntact and ntact <= 16)
  // Split scenes: items run over the workgroup's own frames of the chunk
  // (local frame ofo + X i for own-frame ordinal i = j / ntact).
  const uint32_t inv = 65536u / (uint32_t)(ntact > 0 ? ntact : 1) + 1u;
  int ofo = 0;
  const int own0 = BLK ? lay.own0 : 0;   // (block ownership: BLK builds only)
  auto item_ft = [&](int k, int& fl, int& t) {
    const int j = pw + k * NP;
    const int i = (int)(((uint32_t)j * inv) >> 16);
    t = j - i * ntact;
    fl = ofo + (BLK ? 1 : c.X) * i;
  };
  const brsrc tgr = scene_targets_rsrc(a, s);
  // forward target buffers in flight per producer (4 with 4 producers
  // measured slower: 121 VGPRs, round 4 r4f)
  constexpr int kNB = 2;
  float2 tg[kNB][4] = {};
  auto load_item = [&](int fb, int nitems, int k, float2 (&tg)[4]) {
    const bool ok = k < nitems;
    int fl, t;
    item_ft(ok ? k : 0, fl, t);
    load_targets(tgr, Nmax, c.nact, fb, fl, t, ok, L, q, tg, lay.tfb);
  };
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float lsum = 0.f;
  // the first chunk's staging ahead of the chunk loop: the loop's invariant
  // code (addresses and descriptors for the heads, tiles and errors, which
  // the compiler computes in the loop's preheader) then runs after the
  // staging barriers, not in every producer's prologue before them (there it
  // was ~600 instructions per wave, issued one wave after the other on a
  // SIMD, and the first staging barrier waited for the last)
  if (c.nf > 0) scene_stage<64 * (kRecW + NP), NP, !GRAD, NLL>(a, lay, c, 0, c.nf < lay.fc ? c.nf : lay.fc, [] {});
  for (int fb = 0; fb < c.nf; fb += lay.fc) {
    const int cnt = (c.nf - fb) < lay.fc ? (c.nf - fb) : lay.fc;
    if (fb > 0) {
      scene_pos_dma<64 * (kRecW + NP)>(a, lay, c, fb, cnt);
      scene_stage<64 * (kRecW + NP), NP, !GRAD, NLL>(a, lay, c, fb, cnt, [] {});
    }
    if (fb == 0) act_bits = scene_act_bits(c, scene_mask_word(a, lay, c));   // (the row is in LDS)
    const OwnFrames own = own_frames(fb, cnt, c.X, c.x, own0);
    ofo = own.fo;
    const int nown = INV ? (own.n < 1 ? own.n : 1) : own.n;   // (INV: frame 0 only)
    const int nitems = nown * ntact > pw ? (nown * ntact - pw + NP - 1) / NP : 0;   // forward
    // GRAD: this producer's own frames (ordinals) pw, pw + NP, ... < gend of
    // the chunk (the last R own frames of the last chunk go to the
    // recurrence waves)
    // (INV: producer 0 takes the chunk's frame 0, standing for all cnt)
    const bool live = !BLK || (a.h_in != nullptr && c.x == 0);   // (BLK: does this workgroup run the chain?)
    const int R = GRAD && !INV && fb + lay.fc >= c.nf ? grad_rec_frames(own.n, NP, live) : 0;
    const int gend = INV ? (own.n < 1 ? own.n : 1) : own.n - R;
    // the first tiles' targets: in flight during the heads (GRAD: one buffer
    // and the balancing stores, see grad_frames)
    if (GRAD) {
      load_targets(tgr, Nmax, c.nact, fb, own.fo + (BLK ? 1 : c.X) * pw, 0, pw < gend, L, q, tg[0], lay.tfb);
      balance_stores<PM>(a);
    } else {
#pragma unroll
      for (int j = 0; j < kNB; ++j) load_item(fb, nitems, j, tg[j]);
    }
    float rm[4];
    scene_rm(lay, c, rm);
    // phase 1 — the critical path: frame heads in frame order, As and M into
    // the rings, then the frame's flags; the first heads the recurrence will
    // wait for get the issue priority.  The workgroup running the recurrence
    // forms every frame's head (As), the others only their own frames'; M
    // (and A / cost out) only for own frames.  The recurrence waves form As
    // of the first chunk's frames 0 .. nrh - 1 themselves (M only here).
    const bool all_heads = a.h_in != nullptr && c.x == 0;
    const int hb = all_heads ? 0 : own.fo, hs = all_heads ? 1 : (BLK ? 1 : c.X),
              nh = INV ? (cnt < 1 ? cnt : 1) : (all_heads ? cnt : own.n);   // (INV: one ring slot)
    const int nrep = INV ? cnt : 1;              // frames one head / tile stands for
    const int nrh = all_heads && fb == 0 ? rec_head_frames<CR, INV>(lay, c) : 0;
    for (int i = pw; i < nh; i += NP) {
      const int fl = hb + hs * i;
      const int f = fb + fl;
      const bool mine = !all_heads || c.X == 1 || (BLK ? frame_owner(fb, cnt, fl, c.X, own0) : f % c.X) == c.x;
      if (fl < nrh && (!mine || CR)) continue;   // (a recurrence wave formed As, and M under CR)
      // issue priority: the co-resident geometry is producer-bound, so its
      // producers outrank the chain (2 heads, 3 tiles; round 4,
      // profiles/r4l_prio_ab.txt: eth_hotel_synth 13.4 -> 13.2 us per step);
      // with 12 producers the chain is the critical path
      if (CR) __builtin_amdgcn_s_setprio(2);
      else if (fl >= nrh && fl < NP + nrh) __builtin_amdgcn_s_setprio(1);   // the first round's heads
      const FrameHeadOut hd =
          frame_head<!GRAD, INV>(c.sm, c.sV, c.sVG, fl * stride, lay.wcmax, rm, a.lambda, c.sRing + fl * kD * kD,
                     c.sFlag + fl, f + 1,
                     a.A_out && mine ? a.A_out + ((size_t)s * F + f) * kD * kD : nullptr,
                     a.cost_out && mine ? a.cost_out + ((size_t)s * F + f) * kT * kT : nullptr,
                     GRAD ? c.sCost + fl * kT * kT : nullptr, L, q, mine, fl >= nrh, nrep);
      if (mine) {
        if (L < kL && q < 2) {
          float* m = c.sMring + fl * kL2 * kT;
          *reinterpret_cast<float4*>(m + L * kT + 4 * q) = make_float4(hd.mT0[0], hd.mT0[1], hd.mT0[2], hd.mT0[3]);
          *reinterpret_cast<float4*>(m + (kL + L) * kT + 4 * q) = make_float4(hd.mT1[0], hd.mT1[1], hd.mT1[2], hd.mT1[3]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) lds_store_flag(c.sMflag + fl, f + 1);
      }
      __builtin_amdgcn_s_setprio(0);
    }
    // phase 2 — predictions and errors (GRAD: and the gradient)
    if (CR) __builtin_amdgcn_s_setprio(3);
    if (GRAD) {
      grad_frames<PM, NLL, INV, BLK>(a, lay, c, pw, fb, own.fo + (BLK ? 1 : c.X) * pw, (BLK ? 1 : c.X) * NP, own.fo + (BLK ? 1 : c.X) * gend,
                                act_bits, acc, lsum, tg[0], true, 0, -1, INV ? cnt : 1);
      if (pw < R && grad_rec_tiles(ntact, live) < ntact) {    // the recurrence waves' frames' other tiles
        const int fl = own.fo + (BLK ? 1 : c.X) * (gend + pw);
        grad_frames<PM, NLL, false, BLK>(a, lay, c, pw, fb, fl, 1, fl + 1, act_bits, acc, lsum, tg[0], false,
                             grad_rec_tiles(ntact, live), ntact);
      }
      // every worker done with the chunk's frames -> its dU rows into dV
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) atomicAdd(c.sGseq, 1);
      poll_word(c.sGseq, NP * (fb / lay.fc + 1) + R);    // the recurrence waves add R at the end
      if (ntact > 0) grad_chunk_flush(a, lay, c, fb, cnt, NP);   // (no active pedestrian: all zero)
    } else {
      f32x4 dm[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // (unused by the forward tiles)
      auto item = [&](int k, float2 (&tg)[4]) {
        int fl, t;
        item_ft(k, fl, t);
        const int f = fb + fl;
        poll_flag(c.sMflag + fl, f + 1);         // M of this frame (maybe another producer's)
        const brsrc pr = make_brsrc(a.pred ? a.pred + ((size_t)s * F + f) * kL2 * Nmax : a.targets,
                                    a.pred ? (uint32_t)kL2 * Nmax * 4 : 0u);
        f32x4 dWoT;
        pred_tile<false, PM, false>(c.sMring + fl * kL2 * kT, c.sWo, c.sY, pr, tg,
                                    (act_bits >> t) & 1u, Nmax, c.nact, t, L, q, acc, lsum, dm,
                                    dWoT, [] {});
      };
      if constexpr (INV) {
        auto item_inv = [&](int k, float2 (&tg)[4]) {   // the chunk's frames at once
          int fl, t;
          item_ft(k, fl, t);
          poll_flag(c.sMflag + fl, fb + fl + 1);
          const brsrc pr = make_brsrc(a.pred ? a.pred + ((size_t)s * F + fb) * kL2 * Nmax : a.targets,
                                      a.pred ? (uint32_t)(cnt * kL2 * Nmax * 4) : 0u);
          f32x4 dWoT;
          // (the next item's targets go out once this one's are consumed, ahead
          // of the stores, as in the train tiles)
          pred_tile<false, PM, false, true>(c.sMring + fl * kL2 * kT, c.sWo, c.sY, pr, tg,
                                            (act_bits >> t) & 1u, Nmax, c.nact, t, L, q, acc, lsum, dm,
                                            dWoT, [&] { load_item(fb, nitems, k + 1, tg); }, nullptr,
                                            nullptr, cnt);
        };
        for (int k = 0; k < nitems; ++k) item_inv(k, tg[0]);
      } else {
        for (int k = 0; k < nitems; k += kNB) {
#pragma unroll
          for (int j = 0; j < kNB; ++j) {
            if (k + j < nitems) {
              item(k + j, tg[j]);
              load_item(fb, nitems, k + j + kNB, tg[j]);
            }
          }
        }
      }
    }
    if (CR) __builtin_amdgcn_s_setprio(0);
    if (fb + lay.fc < c.nf) __syncthreads();                    // B3: chunk done (not after the last)
  }
  // metrics (and the loss): GRAD also the recurrence waves' rows (NP + w)
  if (NLL) nll_worker_reduce(c, pw);
  publish_metrics(a, c, pw, GRAD ? NP + kRecW : NP, acc, lsum, GRAD);
  if (!GRAD) return;
  // GRAD: every producer has added its frames once the ticket count is NP;
  // then the scene's gradient row [P + 2] (g2k_weights order) is formed by
  // all producers together
  poll_word(c.sTicket, NP + kRecW);
  grad_priv_sum(c, NP);                                // then all producers see sGAcc
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (lane == 0) atomicAdd(c.sGseq + 1, 1);
  poll_word(c.sGseq + 1, NP);
  const int P = grad_params(Nmax, NLL);
  float* row = a.grad_rows + ((size_t)s * c.X + c.x) * (P + 2);   // this workgroup's row
  const float* ga = c.sGAcc;
  const float* sm = c.sm;
  const int o_wii = Nmax * kD, o_wv = o_wii + kD * kT, o_bv = o_wv + kT * (kD + 2),
            o_wr = o_bv + kD, o_wc = o_wr + kT * 2, o_wo = o_wc + kL2 * kT,
            o_head = o_wo + kT * Nmax;
  // dWi[n][d] = sum_w N[w][n] dV[w][d] + vislet[0][n] dVe[0][d] + vislet[1][n] dVe[1][d]
  // (train.py:76-85 norms of the whole window, re-read from the position rows)
  // by MFMA per 16-pedestrian tile: A[n = L][w] = N[w][n0 + L], B[w][d = L] = dV[w][d]
  const int ntile_all = (Nmax + 15) >> 4;
  #pragma unroll 1
  for (int t = pw; t < ntile_all; t += NP) {
    const int n0 = 16 * t, n = n0 + L;
    f32x4 acc4 = {0.f, 0.f, 0.f, 0.f};
    // one chunk: the whole window is still in LDS (sPos, pitch lay.pp);
    // else the position rows again from global memory.  Two inlined copies,
    // so the LDS one reads by ds_read (one generic pointer for both made
    // them flat loads, counted on vmcnt behind the row's stores)
    auto dwi = [&](const float* prow, int pitch) {
      const int nks = (lay.wtot + 3) / 4;
      const int nc = n < c.nact ? n : 0;
      // four k-steps' position loads in flight (clamped rows, selected after)
#pragma unroll 1
      for (int k0 = 0; k0 < nks; k0 += 4) {
        float2 p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int w = 4 * (k0 + i) + q;
          p[i] = *reinterpret_cast<const float2*>(prow + (size_t)(w < lay.wtot ? w : 0) * pitch + 2 * nc);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int w = 4 * (k0 + i) + q;
          const bool ok = k0 + i < nks && w < lay.wtot;
          const float av = (ok && n < c.nact) ? __builtin_amdgcn_sqrtf(fmaf(p[i].x, p[i].x, p[i].y * p[i].y)) : 0.f;
          const float bv = ok ? c.sGdV[(w < lay.wtot ? w : 0) * kD + L] : 0.f;
          acc4 = mfma4(av, bv, acc4);
        }
      }
    };
    if (n0 < c.nact) {
      if (lay.fc >= F) dwi(c.sPos, lay.pp);
      else dwi(a.pos + (size_t)c.s * a.d.W * Nmax * 2, 2 * Nmax);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int nn = n0 + 4 * q + v;
      if (nn < Nmax) {
        float x = acc4[v];
        if (nn < c.nact)
          x += fmaf(c.sVis[nn], ga[kGA_VE + L], c.sVis[Nmax + nn] * ga[kGA_VE + kD + L]);
        store_wt(row + nn * kD + L, x);
      }
    }
  }
  // the small blocks and dWo, entry by entry over the lanes of the producers
  // without a dWi tile when those are the majority (Nmax 32: six beside the
  // two dWi tiles instead of all eight after them, eth_hotel_synth train
  // 37.8 -> 37.0 us per step; at Nmax 64, four and four, 41.0 -> 41.5: all
  // producers then, as at every larger Nmax).  Each entry is formed by one
  // lane in a fixed order, whichever lane: the same values.
  const int sb0 = 2 * ntile_all < NP ? ntile_all : 0, nsb = NP - sb0;
  if (pw < sb0) return;
  const int ptid = (pw - sb0) * 64 + lane;
  #pragma unroll 1
  for (int p = o_wii + ptid; p < P + 2; p += nsb * 64) {
    float x = 0.f;
    if (p < o_wv) {                                   // dWii[c][u] = sum_t Wv[t][c] AU[t][u]
      const int q2 = p - o_wii, cc = q2 >> 3, uu = q2 & 7;
#pragma unroll
      for (int t = 0; t < kT; ++t) x = fmaf(sm[SM_WV + t * (kD + 2) + cc], ga[kGA_K1 + t * 10 + uu], x);
    } else if (p < o_bv) {                            // dWv
      const int q2 = p - o_wv, t = q2 / (kD + 2), cc = q2 - t * (kD + 2);
      if (cc < kD) {
#pragma unroll
        for (int uu = 0; uu < kT; ++uu) x = fmaf(ga[kGA_K1 + t * 10 + uu], sm[SM_WII + cc * kT + uu], x);
      } else {
        x = ga[kGA_K1 + t * 10 + kT + (cc - kD)];
      }
    } else if (p < o_wr) {
      x = ga[kGA_BV + p - o_bv];
    } else if (p < o_wc) {
      x = 0.f;                                        // Wr does not reach the predictions
    } else if (p < o_wo) {
      x = ga[kGA_WC + p - o_wc];
    } else if (p < o_head) {                          // dWo[t][n]
      const int q2 = p - o_wo, t = q2 / Nmax, nn = q2 - t * Nmax;
      if (lay.dwo_seq) {
        x = c.sGdWo[nn * kT + t];
      } else {
        for (int pr = 0; pr < NP + kRecW; ++pr) x += c.sGdWo[(pr * Nmax + nn) * kT + t];
      }
    } else if (p < P) {                               // NLL head gradient, worker order
      for (int pr = 0; pr < NP + kRecW; ++pr) x += c.sNllW[pr * kNllHead + (p - o_head)];
    } else if (p == P) {                              // loss: 1/2 sum dY^2 (NLL: sum nll), worker order
      for (int pr = 0; pr < NP + kRecW; ++pr) x += c.sMet[pr * 8 + 5];
      x *= NLL ? 1.f : 0.5f;
    } else {                                          // count of (frame, pedestrian) pairs
      for (int pr = 0; pr < NP + kRecW; ++pr) x += c.sMet[pr * 8 + 1];
    }
    store_wt(row + p, x);
  }
}

// GRAD, recurrence wave w after its recurrence: the last R frames of the
// last chunk (frame cnt - R + w) as gradient worker NP + w, then its metrics
// row and ticket (with zero partials when R = 0).
template <int NP, bool PM, bool NLL, bool INV, bool BLK = false>
__device__ __forceinline__ void rec_grad_work(const StepArgs& a, const SceneLayout& lay,
                                              const SceneCtx& c) {
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float lsum = 0.f;
  if (c.nf > 0) {
    const int fb = ((c.nf - 1) / lay.fc) * lay.fc;
    const int cnt = c.nf - fb;
    const OwnFrames own = own_frames(fb, cnt, c.X, c.x, BLK ? lay.own0 : 0);
    const bool live = !BLK || (a.h_in != nullptr && c.x == 0);
    const int R = INV ? 0 : grad_rec_frames(own.n, NP, live);   // (INV: producer 0 has the one frame)
    if (R > 0) {
      float2 tg[4];
      grad_frames<PM, NLL, false, BLK>(a, lay, c, NP + c.wv, fb, own.fo + (BLK ? 1 : c.X) * (own.n - R + c.wv), (BLK ? 1 : c.X) * R,
                           own.fo + (BLK ? 1 : c.X) * own.n,
                           scene_act_bits(c, scene_mask_word(a, lay, c)),
                           acc, lsum, tg, false, 0, grad_rec_tiles(c.ntact, live));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (c.lane == 0) atomicAdd(c.sGseq, 1);
    }
  }
  if (NLL) nll_worker_reduce(c, NP + c.wv);
  publish_metrics(a, c, NP + c.wv, NP + kRecW, acc, lsum, true);
}

// Waves per SIMD the register allocation must leave room for: an 8-wave
// workgroup (NP = 4 below H 512) is sized for two co-resident workgroups per
// CU (4 waves per SIMD, <= 128 VGPRs), so the next launch's scenes start on a
// CU while this launch's recurrence waves finish their chain.
template <int TPW, int NP>
constexpr int scene_waves_per_eu() { return NP == 4 && TPW < 8 ? 4 : 1; }

template <int TPW, int NP, bool GRAD, bool PM, bool NLL, bool INV, bool BLK = false>
__global__ void __launch_bounds__(64 * (kRecW + NP))
__attribute__((amdgpu_waves_per_eu(scene_waves_per_eu<TPW, NP>())))
g2k_scene_kernel(StepArgs a, SceneLayout lay) {
  constexpr int NT = 64 * (kRecW + NP);
  constexpr int kRB = 16 * kRecW;
  // the co-resident geometry (8 waves, two workgroups per CU, forward only):
  // its measured scheduling rules (producer priorities, the recurrence waves'
  // extra heads and M) apply only to it — not to the H = 512 or train-mode
  // 4-producer builds, which run one workgroup per CU
  constexpr bool CR = scene_waves_per_eu<TPW, NP>() > 1 && !GRAD;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  // every kernel-argument line the prologue reads, in ONE scalar-load round
  // trip (left alone, the compiler asks for the n_active / h_in line only
  // after the first batch has landed: a second dependent kernarg miss)
  asm volatile("" ::"s"(a.pos), "s"(a.vislet), "s"(a.G), "s"(a.n_active), "s"(a.n_frames),
               "s"(a.h_in), "s"(a.w.Wi), "s"(a.w.Wo), "s"(a.d.Nmax), "s"(a.d.F), "s"(a.d.W),
               "s"(a.d.stride), "s"(lay.fc), "s"(lay.pp), "s"(lay.o_pos));
  SceneCtx c;
  c.X = lay.split;
  c.s = lay.split == 1 ? (int)blockIdx.x : (int)blockIdx.x / lay.split;
  c.x = (int)blockIdx.x - c.s * lay.split;
  c.tid = threadIdx.x; c.lane = c.tid & 63; c.wv = wave_id(); c.L = c.lane & 15; c.q = c.lane >> 4;
  const int Nmax = a.d.Nmax, F = a.d.F;
  c.ntiles = (Nmax + 15) >> 4;
  c.sWi = smem + lay.o_wi; c.sWo = smem + lay.o_wo; c.sVis = smem + lay.o_vis; c.sV = smem + lay.o_v;
  c.sm = smem + lay.o_small; c.sMet = smem + lay.o_met; c.sRing = smem + lay.o_ring;
  c.sMring = smem + lay.o_mring; c.sRed = smem + lay.o_red; c.sPos = smem + lay.o_pos;
  c.sVG = smem + lay.o_vg;
  c.sFlag = reinterpret_cast<int*>(smem + lay.o_flag);
  c.sMflag = reinterpret_cast<int*>(smem + lay.o_mflag);
  c.sY = smem + lay.o_y;
  c.sTicket = reinterpret_cast<int*>(c.sRed + 2 * kRB) + kRecW;
  c.sCost = smem + lay.o_cost; c.sGFrame = smem + lay.o_gframe;
  c.sGPriv = smem + lay.o_gpriv; c.sGPdV = smem + lay.o_gpdv;
  c.sGAcc = smem + lay.o_gacc;
  c.sGdV = smem + lay.o_gdv; c.sGdWo = smem + lay.o_gdwo;
  c.sGseq = reinterpret_cast<int*>(smem + lay.o_gseq);
  c.sNllA = smem + lay.o_nlla; c.sNllW = smem + lay.o_nllw;
  c.sNllR = smem + lay.o_nllr; c.sNllC = smem + lay.o_nllc;
  if (c.tid <= kRecW) reinterpret_cast<int*>(c.sRed + 2 * kRB)[c.tid] = 0;  // sequence words, ticket
  if (F > 0) {
    // issued before n_active / n_frames arrive: the first chunk's window for
    // min(F, fc) frames (a scene with fewer frames reads rows it ignores)
    const int wv = c.wv, lane = c.lane;
    scene_pos_dma<NT>(a, lay, c, 0, F < lay.fc ? F : lay.fc);   // critical path first
    // the small segments: one wave each (one pointer per wave keeps the
    // kernel-argument loads off a serial s_load / s_waitcnt chain)
    for (int seg = wv; seg < 12; seg += NT / 64) {
      const float* src;
      float* dst;
      int n;
      if (seg == 10 && !NLL) continue;
      if (seg == 11 && !mask_one_load(a)) continue;
      switch (seg) {
        case 0: src = a.w.Wi; dst = c.sWi; n = Nmax * kD; break;
        case 1: src = a.w.Wo; dst = c.sWo; n = kT * Nmax; break;
        case 2: src = a.w.Wii; dst = c.sm + SM_WII; n = kD * kT; break;
        case 3: src = a.G + (size_t)c.s * kD * kT; dst = c.sm + SM_G; n = kD * kT; break;
        case 4: src = a.w.Wv; dst = c.sm + SM_WV; n = kT * (kD + 2); break;
        case 5: src = a.w.bv; dst = c.sm + SM_BV; n = kD; break;
        case 6: src = a.w.Wr; dst = c.sm + SM_WR; n = kT * 2; break;
        case 7: src = a.w.Wc; dst = c.sm + SM_WC; n = kL2 * kT; break;
        case 8: src = a.vislet + (size_t)c.s * 2 * Nmax; dst = c.sVis; n = Nmax; break;
        case 9: src = a.vislet + (size_t)c.s * 2 * Nmax + Nmax; dst = c.sVis + Nmax; n = Nmax; break;
        case 10: src = a.w.head; dst = c.sNllR; n = kNllHead; break;   // NLL head [3][12]
        default:                                       // the ped_mask row, dwords
          src = reinterpret_cast<const float*>(a.ped_mask + (size_t)c.s * Nmax);
          dst = smem + lay.o_mask; n = Nmax / 4; break;
      }
      // 16 bytes per lane when both ends allow it (every segment of the
      // usual layouts): 11 wave-instructions instead of 26 through the CU's
      // vector-memory pipeline, which the whole prologue queues on
      if (((((uintptr_t)src) | lds_addr(dst)) & 15) == 0 && (n & 3) == 0) {
        for (int i = 0; i < n / 4; i += 64)
          if (i + lane < n / 4) dma16(src + 4 * (i + lane), dst + 4 * i);
      } else {
        for (int i = 0; i < n; i += 64)
          if (i + lane < n)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + i + lane),
                                             (__attribute__((address_space(3))) void*)(dst + i), 4, 0, 0);
      }
    }
    if (c.tid < lay.fc) {                                // flags hold (global frame + 1)
      c.sFlag[c.tid] = 0;
      c.sMflag[c.tid] = 0;
    }
  }
  // GRAD: the gradient accumulators and their sequence words zeroed (16 B
  // per lane; the region is 16-B aligned and a multiple of 4 floats) after
  // the prologue's loads are in flight, under their latency (zeroed ahead of
  // the LDS-DMA issue they put it ~4.5k cycles later than a forward launch's)
  auto zero_grad = [&] {
    if (!GRAD) return;
    const int n4 = (lay.o_gseq + rup4(2 + c.ntiles) - lay.o_gacc) >> 2;
    float4* z = reinterpret_cast<float4*>(smem + lay.o_gacc);
    for (int i = c.tid; i < n4; i += NT) z[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.grad_ticket && blockIdx.x == 0 && c.tid == 0) *a.grad_ticket = 0;   // this step's update ticket
  };
  // scene scalars: one scalar round trip (the recurrence's h and the
  // producers' ped_mask word are loaded later, off the prologue's burst)
  auto scalars = [&] {
    int na, nf;
    sload2_i32(a.n_active + c.s, a.n_frames ? a.n_frames + c.s : a.n_active + c.s, na, nf);
    c.nact = clampi(na, 0, Nmax);
    c.nf = a.n_frames ? clampi(nf, 0, F) : F;
    c.ntact = (c.nact + 15) >> 4;                      // tiles holding active pedestrians
    zero_grad();
    if (c.nf == 0) __syncthreads();   // no staging barrier will publish the initialised words
  };
  if (c.wv < kRecW) {
    scalars();
    scene_recurrence<TPW, NP, CR, !GRAD, INV, BLK>(a, lay, c);
    if (GRAD) rec_grad_work<NP, PM, NLL, INV, BLK>(a, lay, c);
  } else {
    scalars();
    scene_producer<NP, GRAD, PM, NLL, CR, INV, BLK>(a, lay, c);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no LDS-DMA outlives the workgroup
}

// Fused scene kernel geometry: producer waves (NP).  Measured (round 1,
// 400 steps): H 256 / Nmax 64: NP 12 28.2 us vs NP 8 29.6; dense crowd
// (H 256, Nmax 256): NP 12 53.2 vs NP 8 60.5; k-fold (H 128, Nmax 64): NP 12
// 23.6 vs NP 8 25.4; eth_hotel_synth (H 128, Nmax 32) then favoured NP 8
// (19.9 vs 20.2), but with this round's cheaper tiles its two-tile scenes are
// producer-bound: NP 12 19.98 vs NP 8 20.75 us (rotated inputs).  So 12
// producers (16 waves, 4 per SIMD) for a lone launch; H = 512 needs > 128
// VGPRs per wave: 4.  Train mode keeps 8 (its producers need more than the
// 128 VGPRs per wave that 16 waves leave).  G2K_STEP_CORESIDENT (launches in
// flight): 4 producers, two 8-wave workgroups per CU when the scene's LDS
// fits twice (round 4, 400 steps over 3-4 streams: eth_hotel_synth 15.5 ->
// 13.5 us per step, kfold4 16.4 -> 11.2, real scenes 16.5 -> 9.3; a lone
// launch 16.0 -> 19.3 us).
int scene_producers(const g2k_dims& d, int H, bool grad) {
  if (H >= 512) return 4;
  if (grad) return 8;
  if (d.flags & G2K_STEP_CORESIDENT) {
    const SceneLayout l = scene_layout(&d, 4, false);
    if ((int64_t)l.total * 4 <= kCoresidentLds) return 4;
  }
  return 12;
}

template <int TPW, int NP, bool GRAD, bool PM>
void launch_kp(const StepArgs& a, const SceneLayout& l, hipStream_t st) {
  const dim3 grid(a.d.S * l.split), block(64 * (kRecW + NP));
  const size_t lds = (size_t)l.total * 4;
  if (GRAD && loss_nll(a.d))
    hipLaunchKernelGGL((g2k_scene_kernel<TPW, NP, GRAD, PM, GRAD, false>), grid, block, lds, st, a, l);
  else if (frames_invariant(a.d, GRAD))   // stride 0, shared targets, one workgroup per scene
    hipLaunchKernelGGL((g2k_scene_kernel<TPW, NP, GRAD, PM, false, true>), grid, block, lds, st, a, l);
  else if (GRAD && l.own0 > 0)           // train, two workgroups per scene: block ownership
    hipLaunchKernelGGL((g2k_scene_kernel<TPW, NP, GRAD, PM, false, false, GRAD>), grid, block, lds, st, a, l);
  else
    hipLaunchKernelGGL((g2k_scene_kernel<TPW, NP, GRAD, PM, false, false>), grid, block, lds, st, a, l);
}

template <int TPW, int NP, bool GRAD>
void launch_k(const StepArgs& a, const SceneLayout& l, hipStream_t st) {
  if (a.d.flags & G2K_STEP_PRED_PED_MAJOR) launch_kp<TPW, NP, GRAD, true>(a, l, st);
  else launch_kp<TPW, NP, GRAD, false>(a, l, st);
}

template <bool GRAD>
int launch_np(const StepArgs& a, const SceneLayout& l, int NP, int tpw, hipStream_t st) {
  if (NP == 4 && tpw == 8) { launch_k<8, 4, GRAD>(a, l, st); return G2K_OK; }
  if constexpr (GRAD) {   // train: NP = 8; forward: NP = 12 (scene_producers)
    if (NP == 8) {
      switch (tpw) {
        case 1: launch_k<1, 8, true>(a, l, st); return G2K_OK;
        case 2: launch_k<2, 8, true>(a, l, st); return G2K_OK;
        case 4: launch_k<4, 8, true>(a, l, st); return G2K_OK;
        default: break;
      }
    }
  } else {
    if (NP == 4) {
      switch (tpw) {
        case 1: launch_k<1, 4, false>(a, l, st); return G2K_OK;
        case 2: launch_k<2, 4, false>(a, l, st); return G2K_OK;
        case 4: launch_k<4, 4, false>(a, l, st); return G2K_OK;
        default: break;
      }
    }
    if (NP == 12) {
      switch (tpw) {
        case 1: launch_k<1, 12, false>(a, l, st); return G2K_OK;
        case 2: launch_k<2, 12, false>(a, l, st); return G2K_OK;
        case 4: launch_k<4, 12, false>(a, l, st); return G2K_OK;
        default: break;
      }
    }
  }
  return set_err(G2K_EUNSUPPORTED, "scene kernel not built for H=%d (NP=%d)", a.d.H, NP);
}

}  // namespace

int64_t scene_lds_bytes(const g2k_dims* d, bool grad) {
  const int H = grad && d->H < 64 ? 64 : d->H;
  return (int64_t)scene_layout(d, scene_producers(*d, H, grad), grad).total * 4;
}

int scene_step_launch(const StepArgs& a, hipStream_t st) {
  const bool grad = a.grad_rows != nullptr;
  // gradient only (no h_in): the recurrence waves idle, the smallest build
  const int H = a.h_in ? a.d.H : 64;
  const int NP = scene_producers(a.d, H, grad);
  const SceneLayout l = scene_layout(&a.d, NP, grad);
  if ((int64_t)l.total * 4 > 160 * 1024)
    return set_err(G2K_ELDS, "Nmax=%d, stride=%d needs %lld bytes of LDS", a.d.Nmax, a.d.stride,
                   (long long)l.total * 4);
  const int tpw = H / 64;
  // split scenes: the scene tickets zeroed on the launch stream first (one
  // 64-byte line per 16 scenes): every launch starts from zero whatever an
  // earlier launch left (an aborted one, a caller's uninitialised workspace)
  if (a.scene_ticket &&
      hipMemsetAsync(a.scene_ticket, 0, (size_t)((a.d.S + 15) / 16) * 64, st) != hipSuccess)
    return set_err(G2K_ELAUNCH, "scene tickets: memset failed");
  const int rc = grad ? launch_np<true>(a, l, NP, tpw, st) : launch_np<false>(a, l, NP, tpw, st);
  if (rc) return rc;
  return check_launch(grad ? "g2k_scene_kernel (train)" : "g2k_scene_kernel");
}

}  // namespace g2k
