/*
 * g2k_hip.h — C ABI of libg2k_hip.so, the MI355X (gfx950) implementation of the
 * g2k_lstm_mcr per-frame path of serenetech90/multimodaltraj_2.
 *
 * The reference has no native plugin API: its boundary is the Python class
 * `g2k_lstm_mcr` plus the TF session feed/fetch protocol.
 * Each entry point below replaces one piece of that boundary; the replaced
 * reference interface is cited per function.  The Python mirror classes in
 * multimodaltraj_2_amd/ bind these through ctypes.
 *
 * Conventions (all entry points):
 *   - every buffer is caller-owned DEVICE memory, contiguous, row-major fp32
 *     unless stated; nullable pointers are marked "or NULL";
 *   - launches are asynchronous on `stream` (a hipStream_t; NULL = default);
 *     no allocation, no host synchronisation: capturable into a hipGraph;
 *   - return 0 on success, a negative G2K_E* code on failure; the message of
 *     the last failure on this thread is in g2k_last_error();
 *   - deterministic: fixed reduction order, no float atomics;
 *   - fixed model geometry: T (obs_len) = 8, L (pred_len) = 12; D = 16
 *     (= neighborhood_size / grid_size, train.py:93) for the fused step and
 *     train mode, D in 1..16 for g2k_mcr_forward_f32 / g2k_frame_recurrence_f32
 *     / g2k_ade_fde_f32 (sample.py runs D = num_freq_blocks = 10,
 *     sample.py:168-205, and the reference checkpoints are D = 10);
 *     H in {64, 128, 256, 512}; Nmax in [1, 256].
 */
#ifndef G2K_HIP_H
#define G2K_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define G2K_ABI_VERSION 9

enum {
  G2K_OK = 0,
  G2K_EINVAL = -1,     /* bad dims / null required pointer */
  G2K_ELAUNCH = -2,    /* HIP launch error */
  G2K_ELDS = -3,       /* requested geometry exceeds LDS */
  G2K_EUNSUPPORTED = -4
};

/* Geometry of one launch (validated on entry). */
typedef struct g2k_dims {
  int32_t S;       /* scenes (batches) in this launch                         */
  int32_t F;       /* frames per scene (max; see n_frames)                    */
  int32_t T;       /* obs_len, must be 8        (argParser.py:26-28)          */
  int32_t L;       /* pred_len, must be 12      (models/g2k_lstm_mcr.py:124)  */
  int32_t D;       /* hidden_len, must be 16    (train.py:93)                 */
  int32_t H;       /* rnn_size                  (argParser.py:8-9)            */
  int32_t Nmax;    /* padded pedestrians per scene                            */
  int32_t W;       /* position rows per scene, >= (F-1)*stride + T            */
  int32_t stride;  /* position-window advance per frame (1 sliding, 0 fixed)  */
  int32_t flags;   /* G2K_STEP_* layout options of the fused step / train mode;
                      0 for every other entry point                           */
} g2k_dims;

/* g2k_dims.flags (g2k_step_fused_f32, g2k_train_step_f32, g2k_step_grad_f32,
 * g2k_step_grad_update_f32):
 *   G2K_STEP_PRED_PED_MAJOR  pred is [S, F, Nmax, L, 2] (pedestrian-major: the
 *     per-pedestrian view the reference's error loops index, pred_path
 *     transposed, train.py:254; the targets' layout) instead of
 *     pred_path_band [S, F, 2L, Nmax]; only pedestrians < n_active are
 *     written (one contiguous n_active * 96-byte run per frame).
 *   G2K_STEP_TARGETS_SHARED  targets is [S, 1, Nmax, L, 2]: one set for every
 *     frame of a scene (the reference feeds a batch's targets to every frame
 *     of its loop, train.py:197-276; real-data scenes). */
#define G2K_STEP_PRED_PED_MAJOR 1
#define G2K_STEP_TARGETS_SHARED 2
/* train mode only: the loss is the bivariate-Gaussian NLL of the prediction
 * pairs around pred with the per-step head w->head (g2k_nll_f32's terms)
 * instead of 1/2 the squared error; the gradient then covers the head too
 * (P = 24 Nmax + 496 + 36, the head's 36 after Wo). */
#define G2K_STEP_LOSS_NLL 4
/* g2k_step_fused_f32 only (the train entry points reject it): the caller keeps
 * two or more launches in flight on separate streams (independent batches).
 * The step is then built from 8-wave workgroups (4 recurrence + 4 producer
 * waves, <= 128 VGPRs, at most half the CU's LDS) so that two of them share a
 * CU: one launch's scenes run while another's recurrence chains finish.  A
 * lone launch is slower this way (fewer producers per scene); the throughput
 * of launches in flight is higher.  When a scene's LDS does not fit twice
 * (e.g. Nmax 256) or H = 512 the usual geometry is used.  The automatic
 * split (below) is 1 under this flag: the launches in flight fill the CUs. */
#define G2K_STEP_CORESIDENT 8
/* Workgroups per scene (bits 8..10): G2K_STEP_SPLIT(x), x in 1..4, or 0 =
 * automatic (x = min(4, CUs / S) for the current device's CU count — 256 on
 * MI355X, 256 assumed without a device — at most F: a launch of fewer scenes
 * than the device has CUs spreads each scene's frames over x workgroups, the
 * first of which also runs the recurrence; g2k_step_split reports x).  The
 * automatic choice is 1 for loop-invariant launches — stride 0 with
 * G2K_STEP_TARGETS_SHARED (and, for the automatic rule, the L2 loss and
 * Nmax <= 85): every frame has the same inputs, and with one workgroup per
 * scene the step forms one frame's head, tiles and gradient terms per chunk
 * and replicates / weights them (pred, h, attn, cost as the general path's;
 * metric sums and gradients n_frames x one frame's).  x > 1
 * needs the workspace (g2k_step_workspace_bytes / g2k_train_workspace_bytes /
 * g2k_grad_workspace_bytes); its contents need no initialisation: every launch
 * zeroes the scene tickets in it on its own stream first (a memset ahead of
 * the kernel), so no earlier call — an aborted one included — can leave state
 * behind.  One workspace per stream: two launches in flight must not share
 * one.  An explicit G2K_STEP_SPLIT(x) makes every size and the launch
 * independent of any device.  With 0 (automatic), the planning calls
 * (g2k_step_split, g2k_*_workspace_bytes) answer for the device current when
 * they are queried (hipGetDevice: they initialise the HIP runtime), while a
 * LAUNCH resolves the automatic choice for the device of the stream it is
 * given (hipStreamGetDevice; the null stream: the current device) and rejects
 * a workspace smaller than that split needs.  Planners that must not depend
 * on the current device ask g2k_step_split_for_cus(d, cus) — host arithmetic,
 * no HIP call — with the CU count of the device they will launch on, and pass
 * the answer as G2K_STEP_SPLIT(x) (ABI 9; what the Python plans do). */
#define G2K_STEP_SPLIT_SHIFT 8
#define G2K_STEP_SPLIT_MASK (7 << G2K_STEP_SPLIT_SHIFT)
#define G2K_STEP_SPLIT(x) ((x) << G2K_STEP_SPLIT_SHIFT)

/* Model parameters (device pointers). Shapes as in the reference. */
typedef struct g2k_weights {
  const float* Wi;   /* [Nmax, D]  weight_input/weight_i   train.py:168-171     */
  const float* Wii;  /* [D, T]     weight_input/weight_ii  train.py:172-175     */
  const float* Wv;   /* [T, D+2]   krnl_weights/weight_v   g2k_lstm_mcr.py:49   */
  const float* bv;   /* [D]        krnl_weights/bias_v     g2k_lstm_mcr.py:55   */
  const float* Wr;   /* [T, 2]     krnl_embed/weight_r     g2k_lstm_mcr.py:72   */
  const float* Wc;   /* [2L, T]    krnl_weights/weight_c   g2k_lstm_mcr.py:65   */
  const float* Wo;   /* [T, Nmax]  krnl_weights/weight_o   g2k_lstm_mcr.py:61   */
  const float* head; /* [3, L] NLL head {log sigma_x, log sigma_y, atanh rho} per
                        step, train mode with G2K_STEP_LOSS_NLL only (else NULL) */
} g2k_weights;

int g2k_abi_version(void);
const char* g2k_last_error(void);

/* Bytes of dynamic LDS per g2k_step_fused_f32 workgroup for `d` (0 if unsupported). */
int64_t g2k_step_lds_bytes(const g2k_dims* d);

/* Bytes of caller-provided device workspace g2k_step_fused_f32 needs for `d`
 * (0: every intermediate stays on chip); -1 on invalid dims. */
int64_t g2k_step_workspace_bytes(const g2k_dims* d);
/* Workgroups per scene the step / train entry points use for `d` (the
 * G2K_STEP_SPLIT request, or the automatic choice); -1 on invalid dims. */
int32_t g2k_step_split(const g2k_dims* d);
/* The automatic split for a device with `cus` compute units (the request when
 * `d` names one; 1 under G2K_STEP_CORESIDENT): host arithmetic only, no HIP
 * call, so a plan can be sized for its device with or without a GPU present;
 * -1 on invalid dims or cus < 1 (ABI 9). */
int32_t g2k_step_split_for_cus(const g2k_dims* d, int32_t cus);
/* Zero-fill `workspace_bytes` bytes of a workspace on `stream` (hipMemsetAsync).
 * (ABI 6 and earlier required it before a split workspace's first use; since
 * ABI 7 every launch zeroes its tickets itself and this is optional.) */
int g2k_workspace_init(void* workspace, int64_t workspace_bytes, void* stream);

/*
 * g2k_step_fused_f32 — the whole per-frame body of train.py:197-276 for S
 * scenes x F frames, one launch:
 *   a2 window norms (train.py:76-85 arithmetic; window = rows f*stride + t),
 *   a3 X0 = Wii @ (Bv @ Wi) (train.py:178-180),
 *   a4 Ve = vislet @ Wi, Rel = Ve*Ve (train.py:182-195),
 *   a7 g2k_lstm_mcr.forward (models/g2k_lstm_mcr.py:99-124),
 *   a8 attention + hidden recurrence (train.py:240-252),
 *   a9 validation ADE/FDE sums (train.py:640-674).
 * Replaces: the frame loop train.py:197-276 (four sess.run + ~13 .eval() per
 * frame) and its per-batch setup train.py:178-195.
 * One launch of the wave-specialised scene kernel (one workgroup per scene:
 * producer waves run a2-a7 / a9 per frame, recurrence waves run a8, LDS flags
 * between them).
 *
 *   pos      [S, W, Nmax, 2]       pedestrian (x, y) rows
 *   vislet   [S, 2, Nmax]          load_traj.py:139 rows 4:6 slice
 *   G        [S, D, T]             `_2dconv_in` feed (train.py:158, 232)
 *   targets  [S, F, Nmax, L, 2]    target assigned to each prediction row
 *                                  ([S, 1, Nmax, L, 2] with G2K_STEP_TARGETS_SHARED)
 *   n_active [S] int32             pedestrians present (<= Nmax)
 *   n_frames [S] int32 or NULL     frames present (<= F); NULL = F
 *   ped_mask [S, Nmax] uint8 or NULL  rows with a target; NULL = all active
 *   h_in     [S, D, H]             hidden_state entering frame 0
 *   h_out    [S, D, H]             hidden_state after the last frame (may alias h_in)
 *   pred     [S, F, 2L, Nmax]      pred_path_band per frame (rows x then y) or, with
 *                                  G2K_STEP_PRED_PED_MAJOR, [S, F, Nmax, L, 2]; only
 *                                  frames < n_frames and columns < min(Nmax,
 *                                  16 ceil(n_active / 16)) are written (whole
 *                                  16-column tiles: the columns past n_active 0)
 *   metrics  [S, 8]                {sum ade_spec, count, sum |fde|^2,
 *                                   sum ade_l2, sum |fde|, frames, 0, 0}
 *   A_out    [S, F, D, D] or NULL  krnl_mdl.attn per frame (frames < n_frames)
 *   cost_out [S, F, T, T] or NULL  krnl_mdl.cost per frame (frames < n_frames)
 *   lambda                          lambda_param (argParser.py, 5e-4)
 *   workspace, workspace_bytes      >= g2k_step_workspace_bytes(d) (may be NULL / 0)
 * h_out must not alias h_in across scenes being read (same-scene aliasing is fine).
 */
int g2k_step_fused_f32(const g2k_dims* d, const g2k_weights* w,
                       const float* pos, const float* vislet, const float* G,
                       const float* targets, const int32_t* n_active,
                       const int32_t* n_frames, const uint8_t* ped_mask,
                       const float* h_in, float* h_out, float* pred,
                       float* metrics, float* A_out, float* cost_out,
                       float lambda, void* workspace, int64_t workspace_bytes,
                       void* stream);

/*
 * g2k_mcr_forward_f32 — g2k_lstm_mcr.forward() for S independent feeds.
 * Replaces: models/g2k_lstm_mcr.py:99-124 and the sess.run at
 * train.py:226-238 (fetches pred_path_band, cost; attn read at :240).
 *   X    [S, D+2, D]  (`outputs` feed)    Rel [S, 2, D] (`rel_features`)
 *   G    [S, D, T]    (`ngh` feed)        n_active [S] int32 (`out_size`)
 *   A_out [S, D, D]   cost_out [S, T, T]  pred [S, 2L, Nmax]
 * Only d->S, T, L, D, Nmax are read.
 */
int g2k_mcr_forward_f32(const g2k_dims* d, const g2k_weights* w,
                        const float* X, const float* Rel, const float* G,
                        const int32_t* n_active, float* A_out, float* cost_out,
                        float* pred, float lambda, void* stream);

/*
 * g2k_frame_embed_f32 — the model input of every frame alone (a2-a4).
 * Replaces: train.py:76-85 (batch_v), 167-180 (inputs = Wii @ (batch_v @ Wi)),
 * 182-195 (vislet_emb, vislet_rel) and the `outputs` feed of :231.
 *   pos [S, W, Nmax, 2], vislet [S, 2, Nmax], n_active [S]; w->Wi [Nmax, D],
 *   w->Wii [D, T] (the other weights are not read)
 *   -> X [S, F, D+2, D] (rows 0..D-1: inputs of frame f's window rows
 *   f*stride + t; rows D, D+1: vislet_emb), Rel [S, 2, D] = vislet_emb^2 or NULL.
 *   D = 16.  The per-frame chain of the --use_grid_lstm encoder stage feeds
 *   the GridLSTM output in place of rows 0..D-1 (multimodaltraj_2_amd/encoder_step.py).
 */
int g2k_frame_embed_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                        const float* vislet, const int32_t* n_active, float* X, float* Rel,
                        void* stream);

/*
 * g2k_frame_recurrence_f32 — attention + hidden-state recurrence of
 * train.py:240-252 over `frames` consecutive attention matrices.
 * Replaces: train.py:240-252 (and its copy at 622-634).
 *   A [S, frames, D, D] (16-byte aligned); h [S, D, H] updated in place.
 *   Reads d->S, D, H.
 */
int g2k_frame_recurrence_f32(const g2k_dims* d, const float* A, float* h,
                             int32_t frames, void* stream);

/*
 * g2k_ade_fde_f32 — displacement errors from predictions.
 *   variant 0: validation sums (train.py:640-674) -> out [S, 8] as metrics above
 *   variant 1: get_mean_error (sample.py:21-82) -> out [S, 8] =
 *              {ADE, FDE, counter, 0...}; pred/targets are [S, 2L, Nmax] /
 *              [S, Nmax, L, 2] with F = 1 and obs_length = d->T.
 * Replaces: the numpy error loops train.py:636-674 and sample.py:21-82.
 *   pred [S, F, 2L, Nmax]; targets [S, F, Nmax, L, 2]; n_active [S];
 *   n_frames [S] or NULL; ped_mask [S, Nmax] or NULL.
 */
int g2k_ade_fde_f32(const g2k_dims* d, const float* pred, const float* targets,
                    const int32_t* n_active, const int32_t* n_frames,
                    const uint8_t* ped_mask, int32_t variant, float* out,
                    void* stream);

/*
 * Elementwise relation ops of nri_learned.py over [rows, cols] matrices.
 * g2k_infer_rlns_f32:  out = sigmoid(adj)           (nri_learned.py:16-21)
 * g2k_eval_rln_ngh_f32: out = softmax(adj, axis=-1) (nri_learned.py:23-28)
 */
int g2k_infer_rlns_f32(const float* adj, float* out, int64_t rows, int32_t cols,
                       void* stream);
int g2k_eval_rln_ngh_f32(const float* adj, float* out, int64_t rows,
                         int32_t cols, void* stream);

/*
 * g2k_gridlstm_f32 — one step of the GridLSTMCell neighbourhood encoders (a6):
 * tf.contrib.rnn.GridLSTMCell(num_units, feature_size, frequency_skip =
 * feature_size, share_time_frequency_weights=True,
 * couple_input_forget_gates=True, state_is_tuple=False), peepholes optional;
 * dataflow decoded from the reference's saved graph.
 * Replaces: helper.py:31-39 + 68 (neighborhood_vis_loc_encoder.forward, with
 * peepholes) and helper.py:131-141 (neighborhood_stat_enc, no peepholes).
 *   in        [rows, ld_in]     frequency block k = columns k*fs .. k*fs+fs-1
 *   state     [rows, ld_state]  block k: c_time = columns 2u*k .. 2u*k+u-1,
 *                               m_time = the next u columns
 *   W [fs + 2u, 3u] (W_f_0_0), b [3u] (B_f_0),
 *   peep [4, u] = (wIf, wIt, wOf, wOt) (W_{I,O}_diag_freq{f,t}_0) or NULL
 *   out       [rows, blocks*2u] = concat_k [m_time', m_freq']
 *   state_out [rows, blocks*2u] = concat_k [c_time', m_time']
 *             (may alias state only when ld_state == blocks*2u)
 * Built for num_units in {1, 2, 4} and feature_size in {2, 4, 8}.
 */
int g2k_gridlstm_f32(const float* in, int64_t ld_in, const float* state, int64_t ld_state,
                     const float* W, const float* b, const float* peep, float* out,
                     float* state_out, int64_t rows, int32_t blocks, int32_t feature_size,
                     int32_t num_units, void* stream);

/*
 * g2k_encoder_chain_f32 — --use_grid_lstm (ABI 8): ONE hidden-state chain
 * through the frames of S batches in order, the vis/loc encoder's
 * GridLSTMCell in every frame (train.py:197-252 with the encoder stage of
 * :201-207 taken as st_embeddings; multimodaltraj_2_amd/encoder_step.py).  ONE
 * workgroup walks the frames (s = 0..S-1, f < n_frames[s]); per frame
 *   Xe[s][f][:D] = GridLSTMCell(X[s][f][:D], h[:, :D])   (as g2k_gridlstm_f32)
 *   attn / cost / pred of that frame from Xe[s][f]       (as g2k_mcr_forward_f32)
 *   h <- one recurrence frame with attn[s][f]            (as g2k_frame_recurrence_f32)
 * bit-identical to those three calls per frame, without a launch per body.
 *   d: S, F, T = 8, L = 12, D = 16, H (64..512), Nmax; W, stride, flags 0
 *   X [S][F][D+2][D], Rel [S][2][D] (g2k_frame_embed_f32), G [S][D][T],
 *   n_active, n_frames [S] (device; n_frames clamped to [0, F]);
 *   cell W [fs + 2u][3u], b [3u], peep [4][u] or NULL, feature_size =
 *   2 num_units (num_units 1, 2, 4: D = 16 columns in, 16 out);
 *   Xe [S][F][D+2][D] out (X copied first; rows 0..D-1 of the run frames
 *   replaced); cell_state [D][D] scratch; attn [S][F][D][D], cost
 *   [S][F][T][T], pred [S][F][2L][Nmax] written for the run frames (others
 *   untouched); h [D][H] in / out (16-byte aligned, as attn).
 */
int g2k_encoder_chain_f32(const g2k_dims* d, const g2k_weights* w, const float* X,
                          const float* Rel, const float* G, const int32_t* n_active,
                          const int32_t* n_frames, const float* cell_W, const float* cell_b,
                          const float* cell_peep, int32_t feature_size, int32_t num_units,
                          float* Xe, float* cell_state, float* attn, float* cost, float* pred,
                          float* h, float lambda, void* stream);

/*
 * Train mode (SURVEY.md §8(d) "--mode train", §8(e) gradient all-reduce).  The
 * reference has no loss or optimizer for this model (SURVEY.md finding 5);
 * these entry points are the build's.  loss = 1/2 the summed squared error of
 * pred_path_band against `targets` over frames < n_frames and the active,
 * masked pedestrians (the pairs the a9 errors use).
 *
 * g2k_grad_size: floats P in one parameter vector = 24*Nmax + 496 (+ 36 with
 *   G2K_STEP_LOSS_NLL), laid out in g2k_weights order (Wi, Wii, Wv, bv, Wr, Wc,
 *   Wo[, head]; padded shapes); -1 on invalid dims.
 * g2k_grad_workspace_bytes: device workspace g2k_step_grad_f32 needs.
 * g2k_step_grad_f32: grad [P + 2] = {d loss / d params summed over the S
 *   scenes (P floats), loss, count of (frame, pedestrian) pairs}, fixed
 *   reduction order (deterministic).  Inputs as g2k_step_fused_f32.  Wr's
 *   gradient is exactly zero (the attention does not reach the predictions).
 * g2k_update_f32: params [P] -= the optimizer step for
 *   g = grad[:P] / max(grad[P+1], 1), clipped by global norm when
 *   grad_clip > 0 (g * clip / max(||g||, clip)), then RMSProp when ms [P] is
 *   given (ms = decay*ms + (1-decay) g^2; p -= lr g / sqrt(ms + 1e-10)) or SGD
 *   (ms NULL).  argParser.py:38-47: grad_clip 10, learning_rate 0.005,
 *   decay_rate 0.95.  Across ranks, all-reduce the [P + 2] grad first.
 */
int64_t g2k_grad_size(const g2k_dims* d);
int64_t g2k_grad_workspace_bytes(const g2k_dims* d);
int g2k_step_grad_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                      const float* vislet, const float* G, const float* targets,
                      const int32_t* n_active, const int32_t* n_frames,
                      const uint8_t* ped_mask, float lambda, float* grad, void* workspace,
                      int64_t workspace_bytes, void* stream);
int g2k_update_f32(float* params, float* ms, const float* grad, int64_t n_params, float lr,
                   float decay, float grad_clip, void* stream);
int64_t g2k_train_workspace_bytes(const g2k_dims* d);
int g2k_train_step_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                       const float* vislet, const float* G, const float* targets,
                       const int32_t* n_active, const int32_t* n_frames,
                       const uint8_t* ped_mask, const float* h_in, float* h_out, float* pred,
                       float* metrics, float lambda, float* grad, void* workspace,
                       int64_t workspace_bytes, float* params, float* ms, float lr, float decay,
                       float grad_clip, void* stream);
/*
 * g2k_train_step_f32: one train-mode step in one call: the fused step's
 *   outputs (h_out, pred, metrics as g2k_step_fused_f32) AND grad [P + 2] from
 *   the same launch (the producers turn each prediction tile's error into the
 *   loss gradient; nothing is recomputed), then the per-scene gradient rows
 *   summed in a fixed order; with params != NULL (one rank) also the update
 *   of g2k_update_f32 (ms NULL: SGD), run by the summing launch's last
 *   workgroup (two launches per step; same results bit for bit as the
 *   separate update).  Across ranks: call with params NULL, all-reduce grad,
 *   then g2k_update_f32.  workspace >= g2k_train_workspace_bytes(d) (one
 *   gradient row per scene and a 64-byte ticket line; no initialisation
 *   needed).
 * g2k_step_grad_update_f32: one rank's whole train-mode update (nothing to
 *   all-reduce): g2k_step_grad_f32 then g2k_update_f32 on params [P] (the flat
 *   buffer in g2k_weights order, P = g2k_grad_size) with the last reduction
 *   pass and the update in one launch.  Same results, bit for bit, as the two
 *   calls; grad [P + 2] is still written.  Same workspace.
 */
int g2k_step_grad_update_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                             const float* vislet, const float* G, const float* targets,
                             const int32_t* n_active, const int32_t* n_frames,
                             const uint8_t* ped_mask, float lambda, float* grad, void* workspace,
                             int64_t workspace_bytes, float* params, float* ms, float lr,
                             float decay, float grad_clip, void* stream);

/*
 * g2k_context_conv_f32 — the static-context input (a5).
 * Replaces: train.py:92-113 (_2dconv = lambda * squeeze(conv2d(pad(img,
 * [[1,1],[0,1],[0,0]]), filter [H+3-D, W+2-D, C, 1], VALID))) and
 * train.py:154-158 (_2dconv_in = _2dconv @ stat_mask, stat_mask [D, T] rows
 * (0, 1/T, ..., (T-1)/T)).
 *   img  [Hh, Ww, C] (HWC, C <= 4)     filt [Hh+3-D, Ww+2-D, C]
 *   out  [D, D] or NULL                 G [D, T = 8] or NULL (one must be set)
 *   D in 1..16; workspace >= g2k_context_conv_workspace_bytes(Hh, Ww, D).
 */
/*
 * Bivariate-Gaussian NLL head and sampling path (the
 * reference has no such head: the build's, parity unpinned — oracle/g2k_ref.py
 * restates it and pins the gradient by central finite differences).
 * head [3][12] = {log sigma_x[t], log sigma_y[t], atanh rho[t]} around
 * mu = pred (pred [S, F, 2L, Nmax] as g2k_step_fused_f32 writes it; targets
 * [S, F, Nmax, L, 2], 8-byte aligned; n_frames / ped_mask may be NULL).
 * g2k_nll_f32: out [38] = {d nll / d head (36, head order), nll summed over
 *   frames < n_frames, active masked pedestrians and the 12 steps, count of
 *   (frame, pedestrian) pairs}, fixed reduction order; dpred (or NULL) =
 *   d nll / d pred for those pairs, zero for the other active columns of
 *   frames < n_frames.  workspace >= g2k_nll_workspace_bytes(d).
 * g2k_gauss_sample_f32: out [S, F, 2L, Nmax] = one draw per (step, pedestrian)
 *   from the head's Gaussian around pred (Box-Muller over a counter-based
 *   hash of seed and the element index: reproducible).  Reads d->S, F, Nmax.
 */
int64_t g2k_nll_workspace_bytes(const g2k_dims* d);
int g2k_nll_f32(const g2k_dims* d, const float* pred, const float* targets,
                const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                const float* head, float* out, float* dpred, void* workspace,
                int64_t workspace_bytes, void* stream);
int g2k_gauss_sample_f32(const g2k_dims* d, const float* pred, const float* head, uint64_t seed,
                         float* out, void* stream);

int64_t g2k_context_conv_workspace_bytes(int32_t Hh, int32_t Ww, int32_t D);
int g2k_context_conv_f32(const float* img, int32_t Hh, int32_t Ww, int32_t C, const float* filt,
                         int32_t D, float lambda, float* out, float* G, void* workspace,
                         int64_t workspace_bytes, void* stream);

/*
 * Tensorized data path (a1/a2 of §8(a)).  Host-side
 * planning (no device memory, callable without a GPU) plus one device gather.
 *
 * g2k_traj_create: index over the columns the frame dict is built from —
 *   `frame` / `ped` are rows 0 / 1 of those columns, `diff` = obs_len.  Keys are
 *   every frame value plus the grid seed + k*diff <= max; grid keys hold their
 *   columns in file order, the others are empty (load_traj.py:234-256
 *   frame_preprocess).  The reference reads the dict from trajectories_0.cpkl
 *   (load_traj.py:95-112), which for every shipped dataset is frame_preprocess
 *   over the WHOLE CSV (the pickles' bytes equal that dict's); eth/univ
 *   has no pickle and is built over the split.  `walk_max` = next_step's bound
 *   max(self.frameList) (load_traj.py:163, 104: the split's, tr_data or
 *   val_data, >= 1).  Returns an opaque handle, NULL on failure.
 *   g2k_traj_destroy frees it.  (ABI 5: `walk_max` added.)
 * g2k_traj_next_step: DataLoader.next_step (load_traj.py:153-224) from
 *   `frame_pointer`: keys[n_keys] = the batch's (non-empty) frame keys in
 *   x_batch order; the target draws as the drawn frames' columns one frame after
 *   the other (draw_cols, draw_len[n_draws] columns per draw; each draw appends
 *   every column pred_len times, quirk Q11); *next_pointer = the advanced
 *   frame_pointer.  draw_cols / draw_len may be NULL.
 * g2k_traj_sample_scenes: for each of n frame pointers, next_step then
 *   ConstructGraph on a fresh graph at framenum 0 with the time slice
 *   (sample.py:138-164; networkx_graph.py:30-73, 114-129): pos_col [n, 8, nmax]
 *   = the CSV column holding node j's position list row t (-1: the zero slot —
 *   a node's first occurrence is not written, rows >= 8 are dropped),
 *   tgt_col [n, nmax, 12] = the columns of node j's first 12 target entries
 *   (-1 past the list), n_nodes [n] = nodes in the graph (may exceed nmax: the
 *   extra nodes are dropped), n_keys [n] = len(batch), next_pointer [n] or NULL.
 *   Node order is the graph's insertion order.
 * g2k_scene_gather_f32: expands those plans on the device: xy [cols, 2] (rows
 *   2:4 of the index's columns, fp32), vis [2, cols] or NULL (rows 4:6; ETH:
 *   none, Q14)
 *   -> pos [S, 8, Nmax, 2] (slot -1: 0), vislet [S, 2, Nmax] = vis[:, vis_off[s]
 *   + n] (train.py:182 / sample.py:184; vis_off NULL = 0), targets
 *   [S, F, Nmax, 12, 2] (the same 12 points for every frame: the reference
 *   feeds one batch's targets to every frame of its loop), ped_mask [S, Nmax]
 *   (1: n < n_active and all 12 target columns present).  Columns >= n_active
 *   are zero.
 */
void* g2k_traj_create(const double* frame, const double* ped, int64_t cols, int32_t diff,
                      double walk_max);
void g2k_traj_destroy(void* traj);
int g2k_traj_next_step(const void* traj, double frame_pointer, int32_t batch_size, int32_t obs_len,
                       double* keys, int32_t max_keys, int32_t* n_keys, int64_t* draw_cols,
                       int64_t max_draw_cols, int64_t* draw_len, int32_t* n_draws,
                       double* next_pointer);
int g2k_traj_sample_scenes(const void* traj, const double* frame_pointers, int32_t n,
                           int32_t batch_size, int32_t obs_len, int32_t pred_len, int32_t nmax,
                           int32_t* pos_col, int32_t* tgt_col, int32_t* n_nodes, int32_t* n_keys,
                           double* next_pointer);
int g2k_scene_gather_f32(const float* xy, const float* vis, int64_t cols, const int32_t* pos_col,
                         const int32_t* tgt_col, const int32_t* vis_off, const int32_t* n_active,
                         int32_t S, int32_t F, int32_t Nmax, float* pos, float* vislet,
                         float* targets, uint8_t* ped_mask, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* G2K_HIP_H */
