// g2k_walk.cpp — the data side of the hot path on the host, natively: the
// reference's DataLoader batch walk (load_traj.py:153-224 next_step) and the
// online graph's scatter into per-node position lists (networkx_graph.py:30-73,
// 114-129), planned for many frame pointers in one call.  The output is index
// plans (CSV column numbers, -1 = the zero slot) that g2k_scene_gather_f32
// expands on the device into the step's [S, ...] tensors.
//
// Semantics are the reference's, including its quirks:
//  * trajectories (load_traj.py:234-256): every frame value of the columns the
//    dict was built over is a key; keys seed + k*diff <= max(frame) hold that
//    frame's rows in file order, the other keys are empty.  The reference READS
//    the dict from trajectories_0.cpkl (load_traj.py:95-112), which for the
//    shipped datasets is frame_preprocess over the WHOLE CSV, while the walk's
//    bound max(self.frameList) (load_traj.py:163) is the split's: the two
//    ranges are separate arguments (`cols` columns, `walk_max`);
//  * next_step: up to batch_size + 1 passes; pass p appends the keys fp, fp +
//    diff, ... (batch_size keys, stopping at the first missing key) to a growing
//    window, then walks the window with one cursor that advances once per
//    visited key and once per target draw; every obs_len-th visit of a
//    non-empty frame draws the frame under the cursor and appends each of its
//    pedestrians' columns pred_len times (Q11); non-empty visited frames form
//    the batch;
//  * ConstructGraph on a FRESH graph (sample.py:150-151): pedestrians without
//    targets are skipped, a pedestrian's first occurrence creates its node
//    with a zero position list (its position is not written), a later
//    occurrence at batch ordinal itr < 8 writes row itr; the node's target is
//    the first 12 entries of its target list (framenum 0).
// Host-only C++ (no device code); part of libg2k_hip.so.
#include <math.h>
#include <stdarg.h>
#include <stdint.h>

#include <climits>

#include <algorithm>
#include <new>
#include <unordered_map>
#include <vector>

#include "g2k_hip.h"

namespace g2k {
int set_err(int code, const char* fmt, ...);
}

namespace {

struct Traj {
  int64_t cols = 0;
  int32_t diff = 8;
  double seed = 0, fmax = 0;                 // the dict's grid: seed .. max over all columns
  double walk_max = 0;                       // next_step's max(self.frameList), :163
  std::vector<int64_t> ped;                  // int(ped id) per column
  std::vector<int32_t> pid;                  // dense pedestrian index per column
  int32_t n_peds = 0;
  std::vector<uint8_t> dup;                  // slot: a pedestrian twice in the frame
  std::unordered_map<double, int32_t> key;   // frame key -> slot
  std::vector<int64_t> beg, end;             // slot -> column range in `rows`
  std::vector<int32_t> rows;                 // columns of each grid key, file order
  int64_t kmin = 0;                          // integer keys: dense slot table
  std::vector<int32_t> islot;

  int32_t slot(int64_t k) const {
    return (k < kmin || k - kmin >= (int64_t)islot.size()) ? -1 : islot[k - kmin];
  }
  int64_t len(int32_t s) const { return end[s] - beg[s]; }
};

struct Plan {        // one next_step call
  std::vector<double> batch;     // non-empty visited keys (x_batch order)
  std::vector<int32_t> bslot;
  std::vector<int32_t> draws;    // slots drawn, in order
  double fp_out = 0;
};

// load_traj.py:153-224
void next_step(const Traj& T, double fp, int bs, int obs, Plan& P) {
  P.batch.clear(); P.bslot.clear(); P.draws.clear();
  std::vector<double> window;
  std::vector<int32_t> wslot;
  // keys lookups are int(fp) + diff*j: membership of the window / batch by j
  const int64_t k0 = (int64_t)fp;
  std::vector<uint8_t> inwin, inbatch;
  auto mark = [&](std::vector<uint8_t>& m, int64_t k) {
    const int64_t j = (k - k0) / T.diff;
    if ((int64_t)m.size() <= j) m.resize(j + 1, 0);
    const bool had = m[j];
    m[j] = 1;
    return had;
  };
  const double lg = log((double)T.diff);
  const double max_idx = T.walk_max;
  const double max_log = log(max_idx) / lg;                     // :166
  double idx = fp;                                              // :167
  int64_t pc = 1;                                               // :162
  for (int b = -1; b < bs;) {                                   // :169
    b += 1;
    double c = max_idx - (idx + 1);                             // :174
    if (c <= 0) break;
    c = log(fabs(c)) / lg;
    if (c <= max_log) {
      const int64_t lo = (int64_t)fp, hi = (int64_t)(fp + (double)bs * obs);   // :182
      for (int64_t k = lo; k < hi; k += T.diff) {               // :184-188
        idx = (double)k;
        const int32_t s = T.slot(k);
        if (s < 0) break;
        if (!mark(inwin, k)) {
          window.push_back((double)k);
          wslot.push_back(s);
        }
      }
      size_t cur = 0;                                           // iter(traj_batch) :190
      for (size_t j = 0; j < window.size(); ++j) {              // :192
        idx = window[j];
        const int32_t s = wslot[j];
        if (T.len(s)) {                                         // :196
          if (!mark(inbatch, (int64_t)idx)) {
            P.batch.push_back(idx);
            P.bslot.push_back(s);
          }
          if (pc % obs == 0) {                                  // :198-213
            if (cur >= window.size()) break;
            P.draws.push_back(wslot[cur++]);
          }
        }
        pc += 1;                                                // :214
        if (cur >= window.size()) break;                        // :215-218
        cur++;
      }
      fp += T.diff;                                             // :220
    } else {
      fp += 8;                                                  // tick_frame_pointer :222
    }
  }
  P.fp_out = fp;
}

// Per-call scratch indexed by dense pedestrian id; `stamp` marks the entries
// that belong to the current scene (no clearing between scenes).
struct Scratch {
  std::vector<int32_t> stamp, cnt, node, cols;
  int32_t gen = 0;
  explicit Scratch(int32_t n) : stamp(n, 0), cnt(n), node(n), cols((size_t)n * 12) {}
  void touch(int32_t p) {
    if (stamp[p] != gen) { stamp[p] = gen; cnt[p] = 0; node[p] = -1; }
  }
};

// sample.py:150-164 on one plan: fresh graph, framenum 0, time slice
void sample_scene(const Traj& T, const Plan& P, int pred_len, int nmax, int32_t* pos_col,
                  int32_t* tgt_col, int32_t* n_nodes, Scratch& W) {
  ++W.gen;
  // each pedestrian's first 12 target entries (the draws, load_traj.py:203-213,
  // rep-major over the frame's rows); with every pedestrian once in the frame
  // a draw adds pred_len copies of its column
  for (int32_t s : P.draws) {
    if (!T.dup[s]) {
      for (int64_t e = T.beg[s]; e < T.end[s]; ++e) {
        const int32_t col = T.rows[e], p = T.pid[col];
        W.touch(p);
        for (int r = 0; r < pred_len && W.cnt[p] < 12; ++r) W.cols[(size_t)p * 12 + W.cnt[p]++] = col;
      }
    } else {
      for (int r = 0; r < pred_len; ++r)
        for (int64_t e = T.beg[s]; e < T.end[s]; ++e) {
          const int32_t col = T.rows[e], p = T.pid[col];
          W.touch(p);
          if (W.cnt[p] < 12) W.cols[(size_t)p * 12 + W.cnt[p]++] = col;
        }
    }
  }
  int32_t P_ = 0;
  for (int i = 0; i < 8 * nmax; ++i) pos_col[i] = -1;
  for (int i = 0; i < 12 * nmax; ++i) tgt_col[i] = -1;
  for (size_t itr = 0; itr < P.bslot.size(); ++itr) {
    const int32_t s = P.bslot[itr];
    for (int64_t e = T.beg[s]; e < T.end[s]; ++e) {
      const int32_t col = T.rows[e], p = T.pid[col];
      if (W.stamp[p] != W.gen) continue;                  // no targets: KeyError, skipped
      if (W.node[p] < 0) {                                // new node: zeros
        const int32_t n = W.node[p] = P_++;
        if (n < nmax)
          for (int l = 0; l < W.cnt[p]; ++l) tgt_col[n * 12 + l] = W.cols[(size_t)p * 12 + l];
      } else if (itr < 8 && W.node[p] < nmax) {           // row itr (IndexError >= 8)
        pos_col[(int)itr * nmax + W.node[p]] = col;
      }
    }
  }
  *n_nodes = P_;
}

}  // namespace

using g2k::set_err;

extern "C" {

void* g2k_traj_create(const double* frame, const double* ped, int64_t cols, int32_t diff,
                      double walk_max) {
  if (!frame || !ped || cols < 1 || diff < 1 || !(walk_max >= 1.0)) {
    set_err(G2K_EINVAL, "g2k_traj_create: bad arguments");
    return nullptr;
  }
  Traj* T = new (std::nothrow) Traj;
  if (!T) {
    set_err(G2K_EINVAL, "g2k_traj_create: out of memory");
    return nullptr;
  }
  T->cols = cols;
  T->diff = diff;
  T->seed = frame[0];                                   // load_traj.py:141
  T->fmax = frame[0];
  T->walk_max = walk_max;
  T->ped.resize(cols);
  T->pid.resize(cols);
  std::unordered_map<int64_t, int32_t> dense;
  for (int64_t i = 0; i < cols; ++i) {
    T->fmax = std::max(T->fmax, frame[i]);
    T->ped[i] = (int64_t)ped[i];                        // int(pedID)
    auto d = dense.emplace(T->ped[i], (int32_t)dense.size()).first;
    T->pid[i] = d->second;
    if (!T->key.count(frame[i])) T->key.emplace(frame[i], (int32_t)T->key.size());
  }
  T->n_peds = (int32_t)dense.size();
  // grid keys seed + k*diff <= max hold their rows (frame_preprocess :247-252)
  std::unordered_map<double, std::vector<int32_t>> grid;
  for (double fp = T->seed; fp <= T->fmax; fp += diff) {
    if (!T->key.count(fp)) T->key.emplace(fp, (int32_t)T->key.size());
    grid.emplace(fp, std::vector<int32_t>());
  }
  for (int64_t i = 0; i < cols; ++i) {
    auto g = grid.find(frame[i]);
    if (g != grid.end()) g->second.push_back((int32_t)i);
  }
  // integer keys (the only ones next_step's int lookups can hit)
  int64_t lo = INT64_MAX, hi = INT64_MIN;
  for (auto& kv : T->key)
    if (kv.first == floor(kv.first) && fabs(kv.first) < 1e15) {
      lo = std::min(lo, (int64_t)kv.first);
      hi = std::max(hi, (int64_t)kv.first);
    }
  if (lo <= hi && hi - lo < (int64_t)1 << 28) {
    T->kmin = lo;
    T->islot.assign(hi - lo + 1, -1);
    for (auto& kv : T->key)
      if (kv.first == floor(kv.first) && fabs(kv.first) < 1e15)
        T->islot[(int64_t)kv.first - lo] = kv.second;
  }
  const size_t ns = T->key.size();
  T->beg.assign(ns, 0);
  T->end.assign(ns, 0);
  T->dup.assign(ns, 0);
  for (auto& kv : T->key) {
    auto g = grid.find(kv.first);
    T->beg[kv.second] = (int64_t)T->rows.size();
    if (g != grid.end()) {
      T->rows.insert(T->rows.end(), g->second.begin(), g->second.end());
      std::vector<int32_t> ids;
      for (int32_t c : g->second) ids.push_back(T->pid[c]);
      std::sort(ids.begin(), ids.end());
      T->dup[kv.second] = std::adjacent_find(ids.begin(), ids.end()) != ids.end();
    }
    T->end[kv.second] = (int64_t)T->rows.size();
  }
  return T;
}

void g2k_traj_destroy(void* h) { delete static_cast<Traj*>(h); }

int g2k_traj_next_step(const void* h, double frame_pointer, int32_t batch_size, int32_t obs_len,
                       double* keys, int32_t max_keys, int32_t* n_keys, int64_t* draw_cols,
                       int64_t max_draw_cols, int64_t* draw_len, int32_t* n_draws,
                       double* next_pointer) {
  const Traj* T = static_cast<const Traj*>(h);
  if (!T || !n_keys || !n_draws || !next_pointer || batch_size < 1 || obs_len < 1)
    return set_err(G2K_EINVAL, "g2k_traj_next_step: bad arguments");
  Plan P;
  next_step(*T, frame_pointer, batch_size, obs_len, P);
  *n_keys = (int32_t)P.batch.size();
  *n_draws = (int32_t)P.draws.size();
  *next_pointer = P.fp_out;
  if ((int64_t)P.batch.size() > max_keys)
    return set_err(G2K_EINVAL, "g2k_traj_next_step: %d keys > max_keys %d", *n_keys, max_keys);
  for (size_t i = 0; i < P.batch.size(); ++i) keys[i] = P.batch[i];
  // the drawn frames' columns, draw after draw (each frame's rows once; the
  // caller repeats them pred_len times, load_traj.py:203-213)
  int64_t n = 0;
  for (size_t i = 0; i < P.draws.size(); ++i) {
    const int32_t s = P.draws[i];
    if (draw_len) draw_len[i] = T->len(s);
    for (int64_t e = T->beg[s]; e < T->end[s]; ++e, ++n)
      if (draw_cols && n < max_draw_cols) draw_cols[n] = T->rows[e];
  }
  if (draw_cols && n > max_draw_cols)
    return set_err(G2K_EINVAL, "g2k_traj_next_step: %lld draw columns > %lld", (long long)n,
                   (long long)max_draw_cols);
  return G2K_OK;
}

int g2k_traj_sample_scenes(const void* h, const double* frame_pointers, int32_t n,
                           int32_t batch_size, int32_t obs_len, int32_t pred_len, int32_t nmax,
                           int32_t* pos_col, int32_t* tgt_col, int32_t* n_nodes,
                           int32_t* n_keys, double* next_pointer) {
  const Traj* T = static_cast<const Traj*>(h);
  if (!T || !frame_pointers || n < 0 || nmax < 1 || batch_size < 1 || obs_len < 1 ||
      pred_len < 1 || !pos_col || !tgt_col || !n_nodes || !n_keys)
    return set_err(G2K_EINVAL, "g2k_traj_sample_scenes: bad arguments");
  Plan P;
  Scratch W(std::max(T->n_peds, 1));
  for (int32_t i = 0; i < n; ++i) {
    next_step(*T, frame_pointers[i], batch_size, obs_len, P);
    sample_scene(*T, P, pred_len, nmax, pos_col + (int64_t)i * 8 * nmax,
                 tgt_col + (int64_t)i * 12 * nmax, n_nodes + i, W);
    n_keys[i] = (int32_t)P.batch.size();
    if (next_pointer) next_pointer[i] = P.fp_out;
  }
  return G2K_OK;
}

}  // extern "C"
