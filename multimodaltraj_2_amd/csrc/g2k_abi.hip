// g2k_abi.hip — the C ABI of libg2k_hip.so (include/g2k_hip.h): argument
// validation, launch planning and the last-error plumbing.  Each entry point
// replaces one piece of the reference's Python/TF boundary (SURVEY.md §8(b);
// the replaced reference interface is cited in the header).
#include <stdarg.h>
#include <stdio.h>

#include "g2k_common.h"

namespace g2k {

namespace {
thread_local char g_err[512] = "";
}

int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int device_cus() {
  // hipDeviceAttributeMultiprocessorCount of the current device, cached per
  // device (256, MI355X's count, when no device is visible: host-only planning)
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    (void)hipGetLastError();
    return 256;
  }
  int n = __atomic_load_n(&cache[dev], __ATOMIC_RELAXED);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) {
    (void)hipGetLastError();
    n = 256;
  }
  __atomic_store_n(&cache[dev], n, __ATOMIC_RELAXED);
  return n;
}

// CUs of the device `st` belongs to (the null stream: the current device);
// 256 when the runtime cannot say
int stream_cus(hipStream_t st) {
  hipDevice_t dev = 0;
  if (st == nullptr || hipStreamGetDevice(st, &dev) != hipSuccess) {
    (void)hipGetLastError();
    return device_cus();
  }
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) {
    (void)hipGetLastError();
    return 256;
  }
  return n;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess)
    return set_err(G2K_ELAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
  return G2K_OK;
}

namespace {

// T, L fixed by the model (argParser.py:26-28, models/g2k_lstm_mcr.py:124);
// D = 16 for the fused step and train mode (train.py:93), 1..16 for the
// class-level forward and the recurrence (sample.py: num_freq_blocks = 10)
int validate_common(const g2k_dims* d, bool need_F, bool any_D = false, int flags_ok = 0) {
  if (!d) return set_err(G2K_EINVAL, "dims is NULL");
  if (d->flags & ~flags_ok)
    return set_err(G2K_EUNSUPPORTED, "flags 0x%x not supported by this entry point", d->flags);
  if (((d->flags & G2K_STEP_SPLIT_MASK) >> G2K_STEP_SPLIT_SHIFT) > kMaxSplit)
    return set_err(G2K_EINVAL, "G2K_STEP_SPLIT(%d): at most %d workgroups per scene",
                   (d->flags & G2K_STEP_SPLIT_MASK) >> G2K_STEP_SPLIT_SHIFT, kMaxSplit);
  if (d->T != kT || d->L != kL)
    return set_err(G2K_EUNSUPPORTED, "unsupported geometry T=%d L=%d (need 8/12)", d->T, d->L);
  if (any_D ? (d->D < 1 || d->D > kD) : d->D != kD)
    return set_err(G2K_EUNSUPPORTED, "unsupported D=%d (%s)", d->D,
                   any_D ? "1..16" : "the fused step needs 16");
  if (d->S < 0) return set_err(G2K_EINVAL, "S=%d < 0", d->S);
  if (d->Nmax < 1 || d->Nmax > kMaxN)
    return set_err(G2K_EINVAL, "Nmax=%d outside [1, %d]", d->Nmax, kMaxN);
  if (need_F && d->F < 0) return set_err(G2K_EINVAL, "F=%d < 0", d->F);
  return G2K_OK;
}

int validate_weights(const g2k_weights* w, bool need_embed) {
  if (!w) return set_err(G2K_EINVAL, "weights is NULL");
  if (!w->Wv || !w->bv || !w->Wr || !w->Wc || !w->Wo)
    return set_err(G2K_EINVAL, "a model weight pointer is NULL");
  if (need_embed && (!w->Wi || !w->Wii)) return set_err(G2K_EINVAL, "Wi/Wii is NULL");
  return G2K_OK;
}

int validate_H(int H) {
  if (H != 64 && H != 128 && H != 256 && H != 512)
    return set_err(G2K_EUNSUPPORTED, "H=%d must be 64, 128, 256 or 512", H);
  return G2K_OK;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// inputs of the fused step (reference and train mode)
int validate_step_inputs(const g2k_dims* d, const g2k_weights* w, const float* pos,
                         const float* vislet, const float* G, const float* targets,
                         const int32_t* n_active, bool train = false) {
  int rc = validate_common(d, true, false,
                           G2K_STEP_PRED_PED_MAJOR | G2K_STEP_TARGETS_SHARED | G2K_STEP_SPLIT_MASK |
                               (train ? G2K_STEP_LOSS_NLL : G2K_STEP_CORESIDENT));
  if (rc) return rc;
  if ((rc = validate_weights(w, true))) return rc;
  if (d->stride < 0) return set_err(G2K_EINVAL, "stride=%d < 0", d->stride);
  if (d->F > 0 && d->W < (d->F - 1) * d->stride + kT)
    return set_err(G2K_EINVAL, "W=%d < (F-1)*stride + T = %d", d->W, (d->F - 1) * d->stride + kT);
  if (!pos || !vislet || !G || !targets || !n_active)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!aligned16(targets)) return set_err(G2K_EINVAL, "targets must be 16-byte aligned");
  if (((uintptr_t)pos & 7u) != 0) return set_err(G2K_EINVAL, "pos must be 8-byte aligned");
  return G2K_OK;
}

// The launch's dims with the split made explicit: an automatic request is
// resolved for the device of the stream the launch goes to (not the current
// device: a plan may be launched on a stream of another device), so every
// later scene_split(a.d) — the workspace check, the kernel layout, the row
// count — agrees with the launch, and a workspace sized for another split is
// rejected by size.
StepArgs step_args(const g2k_dims* d, const g2k_weights* w, const float* pos, const float* vislet,
                   const float* G, const float* targets, const int32_t* n_active,
                   const int32_t* n_frames, const uint8_t* ped_mask, float lambda,
                   hipStream_t st) {
  StepArgs a = {};
  a.d = *d;
  if (split_automatic(a.d))
    a.d.flags |= G2K_STEP_SPLIT(scene_split_cus(a.d, stream_cus(st)));
  a.w = *w; a.pos = pos; a.vislet = vislet; a.G = G; a.targets = targets;
  a.n_active = n_active; a.n_frames = n_frames; a.ped_mask = ped_mask; a.lambda = lambda;
  return a;
}

// [S * X][P + 2] gradient rows (one per workgroup), one 64-byte line for the
// update ticket, then the split workspace (scene tickets, metric partials)
int64_t grad_rows_bytes(const g2k_dims* d) {
  return (int64_t)d->S * scene_split(*d) * (grad_params(d->Nmax, loss_nll(*d)) + 2) * 4 + 64 +
         split_ws_bytes(*d);
}

// train mode after the inputs are validated: the fused step with gradient
// rows into `workspace`, their fixed-order sum into `grad`, the update when
// `params` is given
int train_launch(StepArgs a, float* grad, void* workspace, int64_t workspace_bytes, float* params,
                 float* ms, float lr, float decay, float grad_clip, hipStream_t st) {
  const int width = grad_params(a.d.Nmax, loss_nll(a.d)) + 2;
  if (!grad) return set_err(G2K_EINVAL, "grad is NULL");
  if (loss_nll(a.d) && !a.w.head) return set_err(G2K_EINVAL, "G2K_STEP_LOSS_NLL needs weights->head");
  const int64_t need = grad_rows_bytes(&a.d);
  if (!workspace || workspace_bytes < need)
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed for %d workgroups per scene (got %lld)",
                   (long long)need, scene_split(a.d), (long long)workspace_bytes);
  int rc;
  if (a.d.S == 0 || a.d.F == 0) {
    if (hipMemsetAsync(grad, 0, (size_t)width * 4, st) != hipSuccess)
      return set_err(G2K_ELAUNCH, "train step: memset failed");
    if (a.d.S > 0 && a.h_in && (rc = scene_step_launch(a, st))) return rc;   // forward outputs
    if (params) return update_launch(params, ms, grad, width - 2, lr, decay, grad_clip, st);
    return G2K_OK;
  }
  const int nrows = a.d.S * scene_split(a.d);
  a.grad_rows = static_cast<float*>(workspace);
  int* line = reinterpret_cast<int*>(a.grad_rows + (size_t)nrows * width);
  a.grad_ticket = params ? line : nullptr;
  split_ws_bind(a, line + 16);
  if ((rc = scene_step_launch(a, st))) return rc;
  if (!params) return grad_rows_launch(a.grad_rows, nrows, width, grad, st);
  const UpdateArgs up{params, ms, lr, decay, grad_clip, a.grad_ticket};
  return grad_rows_launch(a.grad_rows, nrows, width, grad, st, &up);
}

}  // namespace
}  // namespace g2k

using namespace g2k;

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int g2k_abi_version(void) { return G2K_ABI_VERSION; }

const char* g2k_last_error(void) { return g_err; }

constexpr int kLayoutFlags = G2K_STEP_PRED_PED_MAJOR | G2K_STEP_TARGETS_SHARED | G2K_STEP_SPLIT_MASK;
constexpr int kStepFlags = kLayoutFlags | G2K_STEP_CORESIDENT;
constexpr int kTrainFlags = kLayoutFlags | G2K_STEP_LOSS_NLL;

int64_t g2k_step_lds_bytes(const g2k_dims* d) {
  if (validate_common(d, true, false, kStepFlags) != G2K_OK) return 0;
  return scene_lds_bytes(d, false);
}

int32_t g2k_step_split(const g2k_dims* d) {
  if (validate_common(d, true, false, kTrainFlags | kStepFlags) != G2K_OK) return -1;
  return scene_split(*d);
}

int32_t g2k_step_split_for_cus(const g2k_dims* d, int32_t cus) {
  if (validate_common(d, true, false, kTrainFlags | kStepFlags) != G2K_OK) return -1;
  if (cus < 1) { set_err(G2K_EINVAL, "cus=%d < 1", cus); return -1; }
  return scene_split_cus(*d, cus);
}

int64_t g2k_step_workspace_bytes(const g2k_dims* d) {
  if (validate_common(d, true, false, kStepFlags) != G2K_OK) return -1;
  return split_ws_bytes(*d);   // one workgroup per scene: every intermediate stays on chip
}

int g2k_workspace_init(void* workspace, int64_t workspace_bytes, void* stream) {
  if (workspace_bytes < 0 || (workspace_bytes > 0 && !workspace))
    return set_err(G2K_EINVAL, "workspace_init: bad arguments");
  if (workspace_bytes == 0) return G2K_OK;
  if (hipMemsetAsync(workspace, 0, (size_t)workspace_bytes, (hipStream_t)stream) != hipSuccess)
    return set_err(G2K_ELAUNCH, "workspace_init: memset failed");
  return G2K_OK;
}

int g2k_step_fused_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                       const float* vislet, const float* G, const float* targets,
                       const int32_t* n_active, const int32_t* n_frames,
                       const uint8_t* ped_mask, const float* h_in, float* h_out, float* pred,
                       float* metrics, float* A_out, float* cost_out, float lambda,
                       void* workspace, int64_t workspace_bytes, void* stream) {
  int rc = validate_step_inputs(d, w, pos, vislet, G, targets, n_active);
  if (rc) return rc;
  if ((rc = validate_H(d->H))) return rc;
  if (!h_in || !h_out || !pred || !metrics)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!aligned16(h_in) || !aligned16(h_out))
    return set_err(G2K_EINVAL, "h_in and h_out must be 16-byte aligned");
  if (workspace_bytes < 0) return set_err(G2K_EINVAL, "negative workspace size");
  if (d->S == 0) return G2K_OK;
  StepArgs a = step_args(d, w, pos, vislet, G, targets, n_active, n_frames, ped_mask, lambda,
                         (hipStream_t)stream);
  const int64_t need = split_ws_bytes(a.d);
  if (need > 0 && (!workspace || workspace_bytes < need))
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed for %d workgroups per scene (got %lld)",
                   (long long)need, scene_split(a.d), (long long)workspace_bytes);
  a.h_in = h_in; a.h_out = h_out; a.pred = pred; a.metrics = metrics; a.A_out = A_out;
  a.cost_out = cost_out;
  split_ws_bind(a, workspace);
  return scene_step_launch(a, (hipStream_t)stream);
}

int64_t g2k_train_workspace_bytes(const g2k_dims* d) {
  if (validate_common(d, true, false, kTrainFlags) != G2K_OK) return -1;
  return grad_rows_bytes(d);
}

int g2k_train_step_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                       const float* vislet, const float* G, const float* targets,
                       const int32_t* n_active, const int32_t* n_frames,
                       const uint8_t* ped_mask, const float* h_in, float* h_out, float* pred,
                       float* metrics, float lambda, float* grad, void* workspace,
                       int64_t workspace_bytes, float* params, float* ms, float lr, float decay,
                       float grad_clip, void* stream) {
  int rc = validate_step_inputs(d, w, pos, vislet, G, targets, n_active, true);
  if (rc) return rc;
  if ((rc = validate_H(d->H))) return rc;
  if (!h_in || !h_out || !pred || !metrics)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!aligned16(h_in) || !aligned16(h_out))
    return set_err(G2K_EINVAL, "h_in and h_out must be 16-byte aligned");
  StepArgs a = step_args(d, w, pos, vislet, G, targets, n_active, n_frames, ped_mask, lambda,
                         (hipStream_t)stream);
  a.h_in = h_in; a.h_out = h_out; a.pred = pred; a.metrics = metrics;
  return train_launch(a, grad, workspace, workspace_bytes, params, ms, lr, decay, grad_clip,
                      (hipStream_t)stream);
}

int g2k_mcr_forward_f32(const g2k_dims* d, const g2k_weights* w, const float* X,
                        const float* Rel, const float* G, const int32_t* n_active, float* A_out,
                        float* cost_out, float* pred, float lambda, void* stream) {
  int rc = validate_common(d, false, true);
  if (rc) return rc;
  if ((rc = validate_weights(w, false))) return rc;
  if (!X || !Rel || !G || !n_active || !A_out || !cost_out || !pred)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (d->S == 0) return G2K_OK;
  return mcr_forward_launch(d, w, X, Rel, G, n_active, A_out, cost_out, pred, lambda,
                            (hipStream_t)stream);
}

int g2k_frame_embed_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                        const float* vislet, const int32_t* n_active, float* X, float* Rel,
                        void* stream) {
  int rc = validate_common(d, true);
  if (rc) return rc;
  if (!w || !w->Wi || !w->Wii) return set_err(G2K_EINVAL, "Wi/Wii is NULL");
  if (d->stride < 0) return set_err(G2K_EINVAL, "stride=%d < 0", d->stride);
  if (d->F > 0 && d->W < (d->F - 1) * d->stride + kT)
    return set_err(G2K_EINVAL, "W=%d < (F-1)*stride + T = %d", d->W, (d->F - 1) * d->stride + kT);
  if (!pos || !vislet || !n_active || !X) return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (((uintptr_t)pos & 7u) != 0) return set_err(G2K_EINVAL, "pos must be 8-byte aligned");
  if ((int64_t)d->S * d->F == 0) return G2K_OK;
  return embed_launch(d, w, pos, vislet, n_active, X, Rel, (hipStream_t)stream);
}

int g2k_frame_recurrence_f32(const g2k_dims* d, const float* A, float* h, int32_t frames,
                             void* stream) {
  if (!d) return set_err(G2K_EINVAL, "dims is NULL");
  if (d->flags) return set_err(G2K_EUNSUPPORTED, "flags must be 0");
  if (d->D < 1 || d->D > kD) return set_err(G2K_EUNSUPPORTED, "D=%d (1..16)", d->D);
  int rc = validate_H(d->H);
  if (rc) return rc;
  if (!A || !h) return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (d->D == kD && (!aligned16(A) || !aligned16(h)))
    return set_err(G2K_EINVAL, "A and h must be 16-byte aligned");
  if (frames < 0 || d->S < 0) return set_err(G2K_EINVAL, "negative frames or S");
  if (d->S == 0) return G2K_OK;
  return recur_launch(A, h, d->S, frames, d->D, d->H, (hipStream_t)stream);
}

int g2k_ade_fde_f32(const g2k_dims* d, const float* pred, const float* targets,
                    const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                    int32_t variant, float* out, void* stream) {
  int rc = validate_common(d, true, true);
  if (rc) return rc;
  if (!pred || !targets || !n_active || !out)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!aligned16(targets)) return set_err(G2K_EINVAL, "targets must be 16-byte aligned");
  if (variant != 0 && variant != 1) return set_err(G2K_EINVAL, "unknown error variant %d", variant);
  if (d->S == 0) return G2K_OK;
  return errors_launch(d, pred, targets, n_active, n_frames, ped_mask, variant,
                       out, (hipStream_t)stream);
}

int g2k_infer_rlns_f32(const float* adj, float* out, int64_t rows, int32_t cols, void* stream) {
  if (!adj || !out || rows < 0 || cols < 0) return set_err(G2K_EINVAL, "bad arguments");
  if (rows * (int64_t)cols == 0) return G2K_OK;
  return relation_launch(adj, out, rows, cols, false, (hipStream_t)stream);
}

int g2k_eval_rln_ngh_f32(const float* adj, float* out, int64_t rows, int32_t cols, void* stream) {
  if (!adj || !out || rows < 0 || cols < 1) return set_err(G2K_EINVAL, "bad arguments");
  if (rows == 0) return G2K_OK;
  return relation_launch(adj, out, rows, cols, true, (hipStream_t)stream);
}

int g2k_gridlstm_f32(const float* in, int64_t ld_in, const float* state, int64_t ld_state,
                     const float* W, const float* b, const float* peep, float* out,
                     float* state_out, int64_t rows, int32_t blocks, int32_t feature_size,
                     int32_t num_units, void* stream) {
  if (!in || !state || !W || !b || !out || !state_out)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (rows < 0 || blocks < 1 || feature_size < 1 || num_units < 1)
    return set_err(G2K_EINVAL, "rows=%lld blocks=%d feature_size=%d num_units=%d", (long long)rows,
                   blocks, feature_size, num_units);
  const int64_t w_out = (int64_t)blocks * 2 * num_units;
  if (ld_in < (int64_t)blocks * feature_size || ld_state < w_out)
    return set_err(G2K_EINVAL, "row pitch too small (ld_in=%lld, ld_state=%lld)", (long long)ld_in,
                   (long long)ld_state);
  if (state_out == state && ld_state != w_out)
    return set_err(G2K_EINVAL, "state_out may alias state only when ld_state == blocks*2*num_units");
  const bool ok_u = num_units == 1 || num_units == 2 || num_units == 4;
  const bool ok_f = feature_size == 2 || feature_size == 4 || feature_size == 8;
  if (!ok_u || !ok_f)
    return set_err(G2K_EUNSUPPORTED, "num_units=%d feature_size=%d (built: units 1/2/4, features 2/4/8)",
                   num_units, feature_size);
  if (rows == 0) return G2K_OK;
  return gridlstm_launch(in, ld_in, state, ld_state, W, b, peep, out, state_out, rows, blocks,
                         feature_size, num_units, (hipStream_t)stream);
}

int g2k_encoder_chain_f32(const g2k_dims* d, const g2k_weights* w, const float* X,
                          const float* Rel, const float* G, const int32_t* n_active,
                          const int32_t* n_frames, const float* cell_W, const float* cell_b,
                          const float* cell_peep, int32_t feature_size, int32_t num_units,
                          float* Xe, float* cell_state, float* attn, float* cost, float* pred,
                          float* h, float lambda, void* stream) {
  int rc = validate_common(d, true);
  if (rc) return rc;
  if ((rc = validate_weights(w, false))) return rc;
  if ((rc = validate_H(d->H))) return rc;
  if (!X || !Rel || !G || !n_active || !n_frames || !cell_W || !cell_b || !Xe || !cell_state ||
      !attn || !cost || !pred || !h)
    return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (!((num_units == 1 && feature_size == 2) || (num_units == 2 && feature_size == 4) ||
        (num_units == 4 && feature_size == 8)))
    return set_err(G2K_EUNSUPPORTED,
                   "num_units=%d feature_size=%d: the encoder maps [D, D] to [D, D] (D = 16) only with "
                   "feature_size = 2 num_units (built: units 1/2/4)", num_units, feature_size);
  if (!aligned16(h) || !aligned16(attn)) return set_err(G2K_EINVAL, "h and attn must be 16-byte aligned");
  if ((int64_t)d->S * d->F == 0) return G2K_OK;
  const hipStream_t st = (hipStream_t)stream;
  if (hipMemcpyAsync(Xe, X, (size_t)d->S * d->F * (kD + 2) * kD * sizeof(float),
                     hipMemcpyDeviceToDevice, st) != hipSuccess)
    return set_err(G2K_ELAUNCH, "Xe: copy of X failed");
  return encoder_chain_launch(d, w, X, Rel, G, n_active, n_frames, cell_W, cell_b, cell_peep,
                              feature_size, num_units, Xe, cell_state, attn, cost, pred, h, lambda, st);
}

int64_t g2k_grad_size(const g2k_dims* d) {
  if (validate_common(d, false, false, kTrainFlags) != G2K_OK) return -1;
  return grad_params(d->Nmax, loss_nll(*d));
}

int64_t g2k_grad_workspace_bytes(const g2k_dims* d) {
  if (validate_common(d, true, false, kTrainFlags) != G2K_OK) return -1;
  return grad_rows_bytes(d);
}

int g2k_step_grad_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                      const float* vislet, const float* G, const float* targets,
                      const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                      float lambda, float* grad, void* workspace, int64_t workspace_bytes,
                      void* stream) {
  int rc = validate_step_inputs(d, w, pos, vislet, G, targets, n_active, true);
  if (rc) return rc;
  StepArgs a = step_args(d, w, pos, vislet, G, targets, n_active, n_frames, ped_mask, lambda,
                         (hipStream_t)stream);
  return train_launch(a, grad, workspace, workspace_bytes, nullptr, nullptr, 0.f, 0.f, 0.f,
                      (hipStream_t)stream);
}

int g2k_step_grad_update_f32(const g2k_dims* d, const g2k_weights* w, const float* pos,
                             const float* vislet, const float* G, const float* targets,
                             const int32_t* n_active, const int32_t* n_frames,
                             const uint8_t* ped_mask, float lambda, float* grad, void* workspace,
                             int64_t workspace_bytes, float* params, float* ms, float lr,
                             float decay, float grad_clip, void* stream) {
  if (!params) return set_err(G2K_EINVAL, "params is NULL");
  int rc = validate_step_inputs(d, w, pos, vislet, G, targets, n_active, true);
  if (rc) return rc;
  StepArgs a = step_args(d, w, pos, vislet, G, targets, n_active, n_frames, ped_mask, lambda,
                         (hipStream_t)stream);
  return train_launch(a, grad, workspace, workspace_bytes, params, ms, lr, decay, grad_clip,
                      (hipStream_t)stream);
}

static int validate_nll(const g2k_dims* d, const float* pred, const float* head,
                        const int32_t* n_active) {
  if (!d) return set_err(G2K_EINVAL, "dims is NULL");
  if (d->flags) return set_err(G2K_EUNSUPPORTED, "flags must be 0 (pred_path_band layout)");
  if (d->T != kT || d->L != kL) return set_err(G2K_EUNSUPPORTED, "T=%d L=%d (8, 12)", d->T, d->L);
  if (d->S < 0 || d->F < 0 || d->Nmax < 1 || d->Nmax > kMaxN)
    return set_err(G2K_EINVAL, "S=%d F=%d Nmax=%d", d->S, d->F, d->Nmax);
  if (!pred || !head || !n_active) return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  return G2K_OK;
}

int64_t g2k_nll_workspace_bytes(const g2k_dims* d) {
  if (!d || d->S < 0) return -1;
  return (int64_t)d->S * (3 * kL + 2) * 4;
}

int g2k_nll_f32(const g2k_dims* d, const float* pred, const float* targets,
                const int32_t* n_active, const int32_t* n_frames, const uint8_t* ped_mask,
                const float* head, float* out, float* dpred, void* workspace,
                int64_t workspace_bytes, void* stream) {
  int rc = validate_nll(d, pred, head, n_active);
  if (rc) return rc;
  if (!targets || !out) return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (((uintptr_t)targets) & 7) return set_err(G2K_EINVAL, "targets must be 8-byte aligned");
  const int64_t need = g2k_nll_workspace_bytes(d);
  if (!workspace || workspace_bytes < need)
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed (got %lld)", (long long)need,
                   (long long)workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  if (d->S == 0) {
    if (hipMemsetAsync(out, 0, (3 * kL + 2) * 4, st) != hipSuccess)
      return set_err(G2K_ELAUNCH, "nll: memset failed");
    return G2K_OK;
  }
  float* rows = static_cast<float*>(workspace);
  if ((rc = nll_launch(d, pred, targets, n_active, n_frames, ped_mask, head, rows, dpred, st)))
    return rc;
  return grad_rows_launch(rows, d->S, 3 * kL + 2, out, st);
}

int g2k_gauss_sample_f32(const g2k_dims* d, const float* pred, const float* head, uint64_t seed,
                         float* out, void* stream) {
  int32_t one = 1;
  int rc = validate_nll(d, pred, head, &one);
  if (rc) return rc;
  if (!out) return set_err(G2K_EINVAL, "out is NULL");
  if ((int64_t)d->S * d->F * kL * d->Nmax == 0) return G2K_OK;
  return gauss_sample_launch(d, pred, head, seed, out, (hipStream_t)stream);
}

int g2k_update_f32(float* params, float* ms, const float* grad, int64_t n_params, float lr,
                   float decay, float grad_clip, void* stream) {
  if (!params || !grad || n_params < 0 || n_params > (1 << 30))
    return set_err(G2K_EINVAL, "bad arguments");
  if (n_params == 0) return G2K_OK;
  return update_launch(params, ms, grad, (int)n_params, lr, decay, grad_clip, (hipStream_t)stream);
}

int64_t g2k_context_conv_workspace_bytes(int32_t Hh, int32_t Ww, int32_t D) {
  if (Hh < 1 || Ww < 1 || D < 1 || D > 16 || Hh + 3 - D < 1 || Ww + 2 - D < 1) return -1;
  return (int64_t)(Hh + 3 - D) * D * D * 4;
}

int g2k_context_conv_f32(const float* img, int32_t Hh, int32_t Ww, int32_t C, const float* filt,
                         int32_t D, float lambda, float* out, float* G, void* workspace,
                         int64_t workspace_bytes, void* stream) {
  if (!img || !filt || (!out && !G)) return set_err(G2K_EINVAL, "a required buffer pointer is NULL");
  if (C < 1 || C > 4) return set_err(G2K_EUNSUPPORTED, "C=%d channels (1..4)", C);
  const int64_t need = g2k_context_conv_workspace_bytes(Hh, Ww, D);
  if (need < 0) return set_err(G2K_EINVAL, "image %dx%d, D=%d (D in 1..16, image >= D)", Hh, Ww, D);
  if (!workspace || workspace_bytes < need)
    return set_err(G2K_EINVAL, "workspace of %lld bytes needed", (long long)need);
  return ctx_conv_launch(img, Hh, Ww, C, filt, D, lambda, out, G, static_cast<float*>(workspace),
                         (hipStream_t)stream);
}

}  // extern "C"
