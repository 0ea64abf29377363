// Context, device memory, streams and the C-ABI of include/kmeans_amd.h.
//
// One km_ctx per GPU (one process per GPU, torch.distributed ranks).  All
// per-iteration work is enqueued on ctx->stream; only calls that hand host
// data back synchronise it.  See DESIGN.md for the data layout in HBM.
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <utility>
#include <vector>

#include "../../include/kmeans_amd.h"
#include "km_internal.h"

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define KM_HIP(call)                                                                               \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess)                                                                          \
      return fail(KM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_) + " (" +           \
                                  std::to_string((int)e_) + ")");                                  \
  } while (0)

#define KM_REQUIRE(cond, code, msg) \
  do {                              \
    if (!(cond)) return fail(code, msg); \
  } while (0)

template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}
template <class T>
void hfree(T*& p) {
  if (p) (void)hipHostFree(p);
  p = nullptr;
}

constexpr int kAllowedDp[] = {16, 32, 48, 64, 96, 128, 192, 256};

// KM_FUSED=0 (diagnostic build only) selects the two-pass MFMA path (screen,
// then a statistics pass) for the shapes the fused kernel covers (A/B runs)
bool fused_disabled() { return km::diag_env("KM_FUSED", 1) == 0; }

// [k][d+1] sums and counts, then the SSE slot
size_t stats_len(const km::Geometry& g) { return (size_t)g.k * (g.d + 1) + 1; }

int choose_dp(int d) {
  for (int v : kAllowedDp)
    if (d <= v) return v;
  return (d + 15) / 16 * 16;  // unsupported by the screening kernels (reported at assign time)
}
}  // namespace

struct km_ctx {
  int device = 0;
  int n_cu = 256;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  km::Geometry g{};
  bool loaded = false;
  bool have_c = false;
  int path = 0;  // 1 small, 2 mfma
  bool fused = false;  // path 2 with the fused assign + sums kernel
  // screen of the fused kernel (km::KM_SCREEN_*), a cost choice (results are
  // exact in every mode), made per batch from the last iteration's queue:
  // fp16x3 with the per-key refinement for the first iteration after new
  // centroids and while more than 1/64 of this rank's rows queue for exact
  // resolution (the refinement costs ~4% where the global test settles
  // nearly every row, and saves most of the exact work where it does not);
  // the fast screen (one fp16 MFMA per product, pairwise bound: 13% less
  // kernel time at c3, ~15-20x the queue) once fewer than 1/2048 of the rows
  // queue, unless it queued more than 1/128 since the last new centroids
  int screen = km::KM_SCREEN_X3_REFINE;
  bool fast_blocked = false;
  int screen_forced = -1;  // km_set_screen: a fixed mode, or -1 (the policy above)
  // one-MFMA screen with in-kernel re-scoring (km_screen1.hip, KM_SCREEN_S1)
  // and delta statistics: where the geometry has an instance, every assign
  // runs k_s1 except the first after new data / centroids / a predict, which
  // runs k_fused16 with full statistics; from then on the stats buffer
  // carries only the moves of rows between clusters, and the update folds
  // them into stats_full (km::launch_s1_apply) before it reads the sums.
  // The choice depends only on the call sequence, never on a rank's data, so
  // every rank of a job takes the same one.
  bool s1 = false;
  // delta statistics on the unfused k_assign_mfma16 geometries as well (c5
  // class: dp a multiple of 32 up to 128): its delta mode writes a change
  // list in its queue layout (chg_m), folded like k_s1's
  bool mdelta_geo = false;
  uint2* chg_m = nullptr;        // k_assign_mfma16 change list [wave][seg] (queue capacity)
  uint32_t* chg_m_cnt = nullptr; // entries per wave
  bool s1_recolor = true;        // colour the chains at the next prep
  int s1_color_age = 0;          // batches since the last colouring
  int s1_batches = 0;            // batches since new centroids
  int32_t* s1_perm = nullptr;    // table index -> centroid
  float* s1_cft = nullptr;       // fp32 centroids by table index (LDS copy)
  float* s1_cn2o = nullptr;      // s^2 ||c||^2, MFMA output order
  uint4* s1_img = nullptr;       // fragment-linear fp16 image of -2 s c
  float* s1_cst = nullptr;       // bound constants
  double* stats_full = nullptr;  // the full sums the deltas apply to
  uint2* chg = nullptr;          // k_s1 change list, one segment per wave, {row, old << 16 | new}
  uint32_t* chg_cnt = nullptr;   // entries per wave segment (written by every delta k_s1)
  bool delta_ready = false;      // labels and stats_full describe one assignment
  bool x3_stale = true;          // Chi/Clo/cn2s/bnd not made for the prepared centroids (ensure_x3)
  bool sweep_rev = false;        // the last k_assign_small / k_s1 launch swept the rows last-first
  int stats_pending = 0;         // the last assign left 0 nothing, 1 full sums, 2 deltas in stats
  bool last_delta = false;       // the last assign with statistics left deltas (km_info.delta_stats)
  bool sse_corr = false;         // the pending SSE slot holds residuals to the fp32 images c' (update corrects)
  float* bal = nullptr;  // fast screen: image error maxima (2 floats)
  // statistics already zero (the batch update cleared them): no memset
  bool stats_clean = false;
  // device repair kernels enqueued in batches: armed for the first batch
  // after new centroids (where empties occur) and after an empty stop;
  // disarmed by a batch without empties (then an empty stops the batch and
  // the host repairs it with the same policy)
  bool rep_armed = false;
  // data
  float* X = nullptr;
  int32_t* labels = nullptr;
  km::QEntry* queue = nullptr;
  uint32_t* qcount = nullptr;
  uint32_t* small_ctr = nullptr;  // small path: queue length, finished workgroups, queued rows (k_assign_small)
  // small path, one rank: km_assign_stats defers its launch and km_update_async
  // launches assign + update as one kernel (the last workgroup updates)
  bool assign_pending = false;
  bool stats_exported = false;  // km_stats_buffer handed the buffer out: a caller may reduce it in between
  uint32_t* cand = nullptr;      // candidate-list pool of the MFMA screen (kind-4 entries)
  uint32_t* cand_ctr = nullptr;  // its per-launch record counter
  uint32_t cand_cap = 0;         // records
  km::QLayout ql{0, 0};
  double* moments = nullptr;  // d+1 scratch
  bool want_sse = false;      // km_set_sse: SSE residuals in km_assign_stats
  int64_t* idx_scratch = nullptr;
  double* rows_scratch = nullptr;
  int64_t scratch_rows = 0;
  // centroids
  int k_alloc = 0;
  double* C64_cur = nullptr;
  double* C64_new = nullptr;
  double* C64T = nullptr;  // transposed [d][k] (full exact scans)
  double* C64P = nullptr;  // padded [kp][dp] (SSE residuals)
  float* C32 = nullptr;
  _Float16* Chi = nullptr;  // fp16 hi/lo of -2*c*s [kp][dp]
  _Float16* Clo = nullptr;
  float* cn2 = nullptr;      // ||c||^2 (fp32)
  float* cn2s = nullptr;     // ||c||^2 s^2, pads 1e30
  float* cmax = nullptr;     // max ||c||
  float* cabs = nullptr;     // max |c_f|
  float* xabs = nullptr;     // max |x_f| over the loaded rows
  float* xnorm = nullptr;    // per-row upper bound of ||x|| (screening bound)
  uint4* ChiF = nullptr;     // fragment-linear hi / lo images (fused kernel)
  uint4* CloF = nullptr;
  float* bnd = nullptr;      // screening-bound constants
  uint32_t* sort_scratch = nullptr;  // label sort of the large-k statistics
  size_t sort_words = 0;
  double* stats_own = nullptr;
  double* stats = nullptr;
  double* work = nullptr;
  int64_t* counts_dev = nullptr;
  km::DevStatus* status_dev = nullptr;
  km::DevStatus* status_host = nullptr;
  int64_t* counts_host = nullptr;
  // batches of iterations without host syncs (km_batch_begin / km_update_async /
  // km_batch_end): per-iteration history, the stop gate every iteration kernel
  // checks, and the centroid buffers each slot read and wrote
  int* gate = nullptr;                 // device: 0 run, KM_STOP_* = stopped
  km::DevStatus* hist = nullptr;       // device [KM_MAX_BATCH]
  km::DevStatus* hist_host = nullptr;  // pinned
  int64_t* hist_counts = nullptr;      // device [KM_MAX_BATCH][k]
  int64_t* hist_counts_host = nullptr; // pinned
  bool in_batch = false;
  int batch_n = 0;
  double* slot_cur[KM_MAX_BATCH] = {};
  double* slot_new[KM_MAX_BATCH] = {};
  // on-device empty-cluster repair (km_set_layout): the dataset's takeSample
  // partition layout and the repair's work buffers
  bool rep_enabled = false;
  int rep_nparts = 0;
  int64_t rep_total = 0, rep_row0 = 0, rep_maxpart = 0;
  int64_t* rep_sizes = nullptr;   // device [nparts]
  int64_t* rep_bases = nullptr;   // device [nparts]
  int rep_cp = 0, rep_k = 0;      // pick slots per partition, k they were sized for
  int32_t* rep_empty = nullptr;   // [k]
  int32_t* rep_pcounts = nullptr; // [nparts]
  int64_t* rep_picks = nullptr;   // [nparts][cp]
  int64_t* rep_samples = nullptr; // [nparts * cp]
  int rep_mode = 0;               // km_set_layout: 1 every row here, 2 rows spread over ranks
  double* rep_rows = nullptr;     // mode 2: replacement rows [k][d], all-reduced by the caller
  double* rep_rows_own = nullptr; // the context's own buffer (unless km_bind_repair_buffer)
  int32_t* rep_pending = nullptr; // mode 2: rows picked by the last k_rep_pick (device word)
  bool rep_wait = false;          // mode 2: km_update_async left the iteration to km_repair_apply_async
  double rep_tol = 0.0;
  bool rep_fold = false;
  // staging
  float* pinned = nullptr;      // two staging halves of pinned_floats each
  size_t pinned_floats = 0;
  hipEvent_t staged[2] = {nullptr, nullptr};  // a half's copy has left it
  // profiling
  int prof = 0;                  // bitmask of KM_K_* phases timed with events
  int prof_period = 1;           // time one launch in prof_period per phase
  int64_t prof_tick[KM_K_COUNT] = {};
  const double* prep_of = nullptr;  // the centroid buffer the derived images were built from
  // timed launches: events, and the batch / slot of the iteration that
  // enqueued them (a stopped batch's later launches are no-ops: km_batch_end
  // drops their timings, so averages count launches that ran)
  struct Timed {
    hipEvent_t first, second;
    int64_t batch;
    int slot;
  };
  std::vector<Timed> ev[KM_K_COUNT];
  int64_t batch_seq = 0;
  std::vector<hipEvent_t> pool;

  hipEvent_t take_event() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    (void)hipEventCreate(&e);
    return e;
  }
};

namespace {

struct ProfScope {
  km_ctx* c;
  int kind;
  bool in_dispatch;  // the events ride in the scope's one timed kernel (KM_TIMED_LAUNCH)
  hipEvent_t a = nullptr, b = nullptr;
  bool on;
  ProfScope(km_ctx* ctx, int k, bool dispatch = false)
      : c(ctx), kind(k), in_dispatch(dispatch),
        on(((c->prof >> k) & 1) && (c->prof_tick[k]++ % c->prof_period) == 0) {
    if (on) {
      a = c->take_event();
      b = c->take_event();
      if (in_dispatch)
        km::g_timing = km::LaunchTiming{a, b};
      else
        (void)hipEventRecord(a, c->stream);
    }
  }
  ~ProfScope() {
    if (on) {
      if (!in_dispatch) {
        (void)hipEventRecord(b, c->stream);
      } else if (km::g_timing.start) {  // no timed launch happened (n = 0): an empty interval
        km::g_timing = km::LaunchTiming{};
        (void)hipEventRecord(a, c->stream);
        (void)hipEventRecord(b, c->stream);
      }
      c->ev[kind].push_back({a, b, c->in_batch ? c->batch_seq : -1, c->batch_n});
    }
  }
};

void free_centroids(km_ctx* c) {
  dfree(c->C64_cur);
  dfree(c->C64_new);
  dfree(c->C64T);
  dfree(c->C64P);
  dfree(c->C32);
  dfree(c->Chi);
  dfree(c->Clo);
  dfree(c->cn2);
  dfree(c->cn2s);
  dfree(c->ChiF);
  dfree(c->CloF);
  dfree(c->bnd);
  c->bal = nullptr;
  dfree(c->cmax);
  dfree(c->cabs);
  dfree(c->stats_own);
  dfree(c->s1_perm);
  dfree(c->s1_cft);
  dfree(c->s1_cn2o);
  dfree(c->s1_img);
  dfree(c->s1_cst);
  dfree(c->stats_full);
  dfree(c->chg);
  dfree(c->chg_cnt);
  c->s1 = false;
  c->mdelta_geo = false;
  c->delta_ready = false;
  c->stats_pending = 0;
  dfree(c->work);
  dfree(c->counts_dev);
  dfree(c->status_dev);
  hfree(c->status_host);
  hfree(c->counts_host);
  dfree(c->hist);
  hfree(c->hist_host);
  dfree(c->hist_counts);
  hfree(c->hist_counts_host);
  c->in_batch = false;
  c->batch_n = 0;
  if (c->stats != nullptr && c->stats != c->stats_own) {
    // external buffer: keep binding only if the size is unchanged (caller re-binds otherwise)
  }
  c->stats = nullptr;
  c->k_alloc = 0;
  c->have_c = false;
}

void free_data(km_ctx* c) {
  dfree(c->X);
  dfree(c->labels);
  dfree(c->queue);
  dfree(c->qcount);
  dfree(c->small_ctr);
  c->assign_pending = false;
  dfree(c->cand);
  dfree(c->cand_ctr);
  c->cand_cap = 0;
  dfree(c->chg_m);
  dfree(c->chg_m_cnt);
  dfree(c->moments);
  dfree(c->xabs);
  dfree(c->xnorm);
  dfree(c->sort_scratch);
  c->sort_words = 0;
  dfree(c->idx_scratch);
  dfree(c->rows_scratch);
  c->scratch_rows = 0;
  c->loaded = false;
  c->delta_ready = false;
}

// derived images (fp32 copy, transposed f64, fp16 hi/lo split, norms, bound
// constants) of centroid buffer `src` (C64_cur, or C64_new speculatively in
// km_update so the next iteration's assign starts right after the host sync)
// the fp16 hi/lo split of the prepared centroid images and the screen's
// bound constants (k_fused16 / k_assign_mfma16 inputs)
int ensure_x3(km_ctx* c) {
  if (!c->x3_stale) return KM_OK;
  KM_HIP(km::launch_prep_split(c->C32, c->g, c->cn2, c->xabs, c->cabs, c->Chi, c->Clo, c->cn2s, c->gate, c->stream));
  KM_HIP(km::launch_bound_consts(c->cmax, c->xabs, c->cabs, c->g, c->bnd, c->gate, c->stream));
  c->x3_stale = false;
  return KM_OK;
}

int prep(km_ctx* c, const double* src) {
  ProfScope ps(c, KM_K_PREP);
  c->prep_of = src;
  if (c->path == 1) {
    KM_HIP(km::launch_prep_small(src, c->g, c->C32, c->cmax, c->gate, c->stream));
    return KM_OK;
  }
  KM_HIP(km::launch_prep_centroids(src, c->g, c->C32, c->cn2, c->cmax, c->cabs, c->C64T, c->C64P, c->gate,
                                   c->stream));
  // the fp16x3 images and screen bounds: k_s1 (and its resolvers) never
  // read them, so with it they are made on first use (ensure_x3)
  c->x3_stale = true;
  if (!c->s1) {
    const int rc = ensure_x3(c);
    if (rc != KM_OK) return rc;
  }
  if (c->s1) {
    if (c->s1_recolor) {
      KM_HIP(km::launch_s1_color(c->C32, c->g, c->s1_perm, c->gate, c->stream));
      c->s1_recolor = false;
    }
    KM_HIP(km::launch_s1_prep(src, c->C32, c->g, c->s1_perm, c->cmax, c->xabs, c->cabs, c->s1_cft, c->s1_cn2o,
                              c->s1_img, c->s1_cst, c->gate, c->stream));
  }
  return KM_OK;
}

int ensure_scratch(km_ctx* c, int64_t rows) {
  if (rows <= c->scratch_rows) return KM_OK;
  dfree(c->idx_scratch);
  dfree(c->rows_scratch);
  KM_HIP(hipMalloc(&c->idx_scratch, sizeof(int64_t) * rows));
  KM_HIP(hipMalloc(&c->rows_scratch, sizeof(double) * rows * std::max(1, c->g.d)));
  c->scratch_rows = rows;
  return KM_OK;
}

int prep(km_ctx* c) { return prep(c, c->C64_cur); }

void free_repair(km_ctx* c) {
  dfree(c->rep_empty);
  dfree(c->rep_pcounts);
  dfree(c->rep_picks);
  dfree(c->rep_samples);
  dfree(c->rep_rows_own);
  dfree(c->rep_pending);
  c->rep_rows = nullptr;
  c->rep_cp = 0;
  c->rep_k = 0;
}

// takeSample's fraction for num rows of total (sampling.py _fraction)
double sample_fraction(int64_t num, int64_t total) {
  const double fraction = (double)num / (double)total;
  const double gamma = -std::log(0.00005) / (double)total;
  return std::min(1.0, fraction + gamma + std::sqrt(gamma * gamma + 2.0 * gamma * fraction));
}

// repair buffers sized for the largest repair (all k clusters empty): per
// partition 4x the expected picks + 64 slots (more -> the host repairs)
int ensure_repair(km_ctx* c) {
  if (c->rep_k == c->g.k && c->rep_pcounts) return KM_OK;
  free_repair(c);
  const double f = sample_fraction(std::min<int64_t>(c->g.k, std::max<int64_t>(c->rep_total - 1, 1)),
                                   std::max<int64_t>(c->rep_total, 1));
  const double cpd = 4.0 * f * (double)c->rep_maxpart + 64.0;
  KM_REQUIRE(cpd < (double)(1 << 26), KM_ERR_ARG, "km_update_async: repair buffers too large");
  c->rep_cp = (int)cpd;
  const size_t slots = (size_t)c->rep_cp * c->rep_nparts;
  KM_HIP(hipMalloc(&c->rep_empty, sizeof(int32_t) * c->g.k));
  KM_HIP(hipMalloc(&c->rep_pcounts, sizeof(int32_t) * c->rep_nparts));
  KM_HIP(hipMemsetAsync(c->rep_pcounts, 0, sizeof(int32_t) * c->rep_nparts, c->stream));
  KM_HIP(hipMalloc(&c->rep_picks, sizeof(int64_t) * slots));
  KM_HIP(hipMalloc(&c->rep_samples, sizeof(int64_t) * slots));
  KM_HIP(hipMalloc(&c->rep_pending, sizeof(int32_t)));
  KM_HIP(hipMemsetAsync(c->rep_pending, 0, sizeof(int32_t), c->stream));
  if (c->rep_mode == 2) {
    KM_HIP(hipMalloc(&c->rep_rows_own, sizeof(double) * (size_t)c->g.k * std::max(1, c->g.d)));
    c->rep_rows = c->rep_rows_own;
  }
  c->rep_k = c->g.k;
  return KM_OK;
}

// the small path's queue (the QEntry queue's storage as row indices: its
// capacity holds n of them) and counters; no update folded in
// serpentine sweeps: where X is at most 8 GiB, alternate launches of the
// streaming screens visit the rows last-first, so each starts on the rows
// the last one read last, still in the 256 MiB Infinity Cache (c2 640 MB:
// +6%; c3_shard8 3.2 GB: +2%).  Larger X gains nothing from the cache and
// the descending sweep measured 2-3% slower at c3 (25.6 GB), so it stays
// ascending there
bool next_sweep(km_ctx* c) {
  if ((double)c->g.n * c->g.dp * 4.0 > 8.0 * (1ull << 30)) return false;
  c->sweep_rev = !c->sweep_rev;
  return c->sweep_rev;
}

km::SmallTail small_tail(km_ctx* c) {
  km::SmallTail t{};
  t.queue = reinterpret_cast<uint32_t*>(c->queue);
  t.qctr = c->small_ctr;
  t.done = c->small_ctr + 1;
  t.kp = c->g.kp;
  t.qout = c->qcount;
  t.rev = next_sweep(c);
  return t;
}

// the update folds into the assign launch: small path, one workgroup update,
// the context's own statistics (no caller reduces them between assign and
// update), no device repair behind it
bool fold_ok(km_ctx* c) {
  return c->in_batch && c->path == 1 && km::update_one_ok(c->g) && c->stats == c->stats_own && !c->stats_exported &&
         !(c->rep_enabled && c->rep_armed);
}

int run_assign(km_ctx* c, bool with_stats);

// the one-MFMA unfused screen re-scores its pairs in fp32 in the kernel (A/B
// knob: 0 leaves them all to k_rerank2)
#ifndef KM_PAIR_RESCORE
#define KM_PAIR_RESCORE 1
#endif

// the unfused screen with one fp16 MFMA per product (KM_SCREEN_ONE): forced,
// or by default where k_s1 has no instance (dp a multiple of 32, <= 256)
bool one_screen(km_ctx* c) {
  if (c->path != 2 || c->fused || c->g.dp % 32 != 0 || c->g.dp > 256) return false;
  if (c->screen_forced == KM_SCREEN_ONE) return true;
  return c->screen_forced < 0 && !c->s1;
}

// k_s1 for this assign: labels only (predict), or delta statistics once the
// labels and the full sums of a previous iteration are in place (with
// compute_sse k_s1 also adds every row's residual to the fp32 image of its
// centroid, the resolvers the queued rows', and the update corrects the total
// to the exact SSE: every row is read once either way)
bool use_s1(km_ctx* c, bool with_stats) {
  if (!c->s1) return false;
  if (c->screen_forced >= 0 && c->screen_forced != KM_SCREEN_S1) return false;
  // (a caller that took the buffer with km_stats_buffer reads full sums)
  return !with_stats || (c->delta_ready && !c->stats_exported && km::s1_delta_ok(c->g, c->n_cu));
}

// before an update reads the statistics: delta -> fold into the full sums;
// full -> keep them as the base of the next deltas.  Returns the buffer the
// update reads: with `clear` (an update that leaves its input alone) the
// folded sums stay in stats_full and the deltas are zeroed for the next
// iteration (no memset before it); else stats = the folded sums.
int apply_stats(km_ctx* c, const double** upd_src = nullptr, bool clear = false) {
  const int kind = c->stats_pending;
  c->stats_pending = 0;
  if (upd_src) *upd_src = c->stats;
  if (!c->s1 && !c->mdelta_geo) return KM_OK;
  // full sums (kind 1) become the base of the next deltas, the deltas
  // (kind 2) are folded into them (k_s1_apply replaces the SSE slot)
  const bool keep = kind == 2 || kind == 1;
  const bool zero = kind == 2 && clear && upd_src;
  if (keep)
    KM_HIP(km::launch_s1_apply(c->stats, c->stats_full, (int64_t)stats_len(c->g), kind == 2 ? (zero ? 2 : 1) : 0,
                               c->gate, c->stream));
  if (zero) {
    *upd_src = c->stats_full;
    c->stats_clean = true;  // the deltas are zero for the next assign
  }
  c->delta_ready = keep;
  return KM_OK;
}

// the SSE correction flag of the statistics an update is about to read
// (consumed once)
int take_sse_corr(km_ctx* c) {
  const bool v = c->sse_corr;
  c->sse_corr = false;
  return v ? 1 : 0;
}

// a deferred km_assign_stats launched on its own (any call but km_update_async
// that follows it)
int flush_assign(km_ctx* c) {
  if (!c->assign_pending) return KM_OK;
  c->assign_pending = false;
  return run_assign(c, true);
}

int run_assign(km_ctx* c, bool with_stats) {
  const km::Geometry& g = c->g;
  if (c->prep_of != c->C64_cur) {
    const int rc = prep(c);
    if (rc != KM_OK) return rc;
  }
  c->ql = km::QLayout{0, 0};
  if (with_stats && c->stats_pending == 2) {
    // a second km_assign_stats before the update: the first one's labels are
    // in place but its deltas were never folded into stats_full, so the
    // deltas against those labels would describe the wrong base; this pass
    // computes full sums instead (the same choice on every rank: it depends
    // on the call sequence only)
    c->delta_ready = false;
  }
  const bool sse = with_stats && c->want_sse;
  double* sse_slot = c->stats + (size_t)g.k * (g.d + 1);
  if (with_stats && !c->stats_clean) KM_HIP(hipMemsetAsync(c->stats, 0, sizeof(double) * stats_len(g), c->stream));
  if (with_stats) c->stats_clean = false;
  if (c->path == 1) {
    ProfScope ps(c, KM_K_ASSIGN, true);
    KM_HIP(km::launch_assign_small(c->X, g, c->C32, c->C64_cur, c->cmax, c->labels, c->stats, with_stats ? 1 : 0,
                                   sse ? 1 : 0, c->n_cu, c->gate, c->stream, small_tail(c)));
    c->ql = km::QLayout{0, g.n > 0 ? 1u : 0u};  // its last workgroup leaves the queued rows in qcount[0]
    return KM_OK;
  }
  // (a predict between an assign and its update leaves that assign's
  // statistics pending: the update still folds them)
  if (with_stats) {
    c->stats_pending = 1;
    c->last_delta = false;
    c->sse_corr = false;
  }
  if (use_s1(c, with_stats)) {
    // compute_sse with delta statistics: residuals to the fp32 images c'
    // (k_s1, the resolvers), corrected by the update (km::launch_update corr)
    double* s1_sse = sse ? sse_slot : nullptr;
    {
      ProfScope ps(c, KM_K_ASSIGN, true);
      KM_HIP(km::launch_s1(c->X, c->xnorm, g, c->s1_img, c->s1_cn2o, c->s1_cft, c->s1_perm, c->s1_cst,
                           c->labels, c->queue, c->qcount, c->chg, c->chg_cnt, with_stats ? 1 : 0, c->n_cu,
                           &c->ql, c->gate, c->stream, next_sweep(c), s1_sse));
    }
    {
      // the queued rows: near-ties of the re-scored candidates and the rows
      // the chain certificate leaves open, resolved in float64 (delta: they
      // still hold their previous labels)
      ProfScope ps(c, KM_K_RESOLVE);
      KM_HIP(km::launch_resolve(c->X, g, c->C64_cur, c->C64T, c->queue, c->qcount, c->ql, c->labels, nullptr,
                                c->n_cu, c->gate, c->stream, s1_sse, nullptr, 0, with_stats ? 1 : 0,
                                s1_sse ? c->C32 : nullptr, c->chg, c->chg_cnt, c->C32, c->cmax));
    }
    if (with_stats) {
      // the rows k_s1 moved between clusters (its change list) into the deltas
      ProfScope ps(c, KM_K_STATS);
      KM_HIP(km::launch_s1_delta(c->X, g, c->chg, c->chg_cnt, c->stats, c->n_cu, c->gate, c->stream, c->qcount));
    }
    if (with_stats) {
      c->stats_pending = 2;
      c->last_delta = true;
      c->sse_corr = s1_sse != nullptr;
    }
    return KM_OK;
  }
  if (c->fused) {
    {
      const int rc = ensure_x3(c);
      if (rc != KM_OK) return rc;
    }
    {
      ProfScope ps(c, KM_K_ASSIGN, true);
      KM_HIP(km::launch_fused(c->X, c->xnorm, g, c->Chi, c->Clo, c->ChiF, c->CloF, c->cn2s, c->bnd, c->xabs, c->cabs,
                              c->labels, c->queue, c->qcount, c->stats, with_stats ? 1 : 0,
                              (with_stats || c->screen >= km::KM_SCREEN_FAST1) ? c->screen : km::KM_SCREEN_X3_REFINE,
                              c->n_cu, &c->ql, c->gate, c->stream, c->C32, c->cmax, c->bal, c->C64P,
                              sse ? sse_slot : nullptr));
    }
    {
      // SSE: the fused kernel adds every decided row's residual, the
      // resolvers the queued rows' (same pass, no second read of X)
      ProfScope ps(c, KM_K_RESOLVE);
      KM_HIP(km::launch_resolve(c->X, g, c->C64_cur, c->C64T, c->queue, c->qcount, c->ql, c->labels,
                                with_stats ? c->stats : nullptr, c->n_cu, c->gate, c->stream,
                                sse ? sse_slot : nullptr, nullptr, 0, 0, nullptr, nullptr, nullptr, c->C32, c->cmax));
    }
    return KM_OK;  // counts are part of the fused and resolver statistics
  }
  if (c->s1 && !c->fused && (c->screen_forced < 0 || c->screen_forced == KM_SCREEN_S1)) {
    // unfused geometry (c4 class): k_s1's labels (queued rows resolved in
    // float64), then the statistics pass below reads X once more
    {
      ProfScope ps(c, KM_K_ASSIGN, true);
      KM_HIP(km::launch_s1(c->X, c->xnorm, g, c->s1_img, c->s1_cn2o, c->s1_cft, c->s1_perm, c->s1_cst, c->labels,
                           c->queue, c->qcount, c->chg, c->chg_cnt, 0, c->n_cu, &c->ql, c->gate, c->stream,
                           next_sweep(c)));
    }
    {
      ProfScope ps(c, KM_K_RESOLVE);
      KM_HIP(km::launch_resolve(c->X, g, c->C64_cur, c->C64T, c->queue, c->qcount, c->ql, c->labels, nullptr,
                                c->n_cu, c->gate, c->stream, nullptr, nullptr, 0, 0, nullptr, nullptr, nullptr, c->C32,
                                c->cmax));
    }
  } else {
  if (!c->cand && g.dp <= 256) {
    // candidate lists of the points the screen cannot settle between its top
    // two (kind 4): up to 4M records of 64 B; a full pool leaves the rest to
    // the full scans
    const int64_t cap = std::min<int64_t>(std::max<int64_t>(g.n, 1024), (int64_t)1 << 22);
    KM_HIP(hipMalloc(&c->cand, sizeof(uint32_t) * km::cand_rec_words() * (size_t)cap));
    KM_HIP(hipMalloc(&c->cand_ctr, sizeof(uint32_t)));
    c->cand_cap = (uint32_t)cap;
  }
  {
    const int rc = ensure_x3(c);
    if (rc != KM_OK) return rc;
  }
  // delta statistics (c5 class, no SSE): the screen lists the rows whose
  // label changed, the resolvers move their changed rows, and the change list
  // is folded into the deltas -- no statistics pass over X
  const bool mdelta = with_stats && c->mdelta_geo && c->delta_ready && !c->want_sse && !c->stats_exported;
  if (mdelta && !c->chg_m) {
    KM_HIP(hipMalloc(&c->chg_m, sizeof(uint2) * km::queue_capacity(std::max<int64_t>(g.n, 1), c->n_cu)));
    KM_HIP(hipMalloc(&c->chg_m_cnt, sizeof(uint32_t) * km::qcount_words(c->n_cu)));
  }
  {
    ProfScope ps(c, KM_K_ASSIGN);
    KM_HIP(km::launch_assign_mfma(c->X, g, c->Chi, c->Clo, c->cn2s, c->cmax, c->xabs, c->cabs, c->labels, c->queue,
                                  c->qcount, c->n_cu, &c->ql, c->gate, c->stream, c->cand, c->cand_ctr,
                                  c->cand_cap, one_screen(c) ? 1 : 0, KM_PAIR_RESCORE ? c->C32 : nullptr,
                                  mdelta ? c->chg_m : nullptr, mdelta ? c->chg_m_cnt : nullptr));
  }
  {
    ProfScope ps(c, KM_K_RESOLVE);
    KM_HIP(km::launch_resolve(c->X, g, c->C64_cur, c->C64T, c->queue, c->qcount, c->ql, c->labels, nullptr, c->n_cu,
                              c->gate, c->stream, nullptr, c->cand, c->cand_cap, mdelta ? 1 : 0, nullptr,
                              mdelta ? c->chg_m : nullptr, mdelta ? c->chg_m_cnt : nullptr, c->C32, c->cmax));
  }
  if (mdelta) {
    ProfScope ps(c, KM_K_STATS);
    KM_HIP(km::launch_chg_delta(c->X, g, c->chg_m, c->chg_m_cnt, (int)c->ql.nwaves, c->ql.seg, c->stats, c->n_cu,
                                c->gate, c->stream, c->qcount));
    c->stats_pending = 2;
    c->last_delta = true;
    return KM_OK;
  }
  }
  if (with_stats) {
    ProfScope ps(c, KM_K_STATS);
    if (km::stats_needs_sort(g)) {
      const size_t words = km::sorted_stats_words(g.n, g.k);
      if (words > c->sort_words) {
        dfree(c->sort_scratch);
        KM_HIP(hipMalloc(&c->sort_scratch, sizeof(uint32_t) * words));
        c->sort_words = words;
      }
      KM_HIP(km::launch_stats_sorted(c->X, g, c->labels, c->stats, c->sort_scratch, sse ? c->C64P : nullptr,
                                     c->n_cu, c->gate, c->stream));
    } else {
      // SSE residuals in the same pass over X (feature-range tiles)
      KM_HIP(km::launch_stats(c->X, g, c->labels, c->stats, c->n_cu, c->gate, c->stream, sse ? c->C64P : nullptr,
                              sse ? c->C32 : nullptr));
    }
  }
  return KM_OK;
}

}  // namespace

extern "C" {

int km_abi_version(void) { return KM_ABI_VERSION; }

const char* km_last_error(void) { return g_err.c_str(); }

int km_device_count(int* out) {
  KM_REQUIRE(out, KM_ERR_ARG, "km_device_count: null out");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) n = 0;
  *out = n;
  return KM_OK;
}

int km_create(int device, km_ctx** out) {
  KM_REQUIRE(out, KM_ERR_ARG, "km_create: null out");
  *out = nullptr;
  int n = 0;
  KM_HIP(hipGetDeviceCount(&n));
  KM_REQUIRE(device >= 0 && device < n, KM_ERR_ARG,
             "km_create: device " + std::to_string(device) + " out of range (" + std::to_string(n) + " devices)");
  KM_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  KM_HIP(hipGetDeviceProperties(&prop, device));
  KM_REQUIRE(std::string(prop.gcnArchName).rfind("gfx950", 0) == 0, KM_ERR_UNSUPPORTED,
             std::string("km_create: kernels are built for gfx950 (MI355X), device is ") + prop.gcnArchName);
  km_ctx* c = new km_ctx();
  c->device = device;
  c->n_cu = prop.multiProcessorCount;
  hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return fail(KM_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  c->stream = c->own_stream;
  e = hipMalloc(&c->gate, sizeof(int));
  if (e == hipSuccess) e = hipMemset(c->gate, 0, sizeof(int));
  if (e != hipSuccess) {
    (void)hipStreamDestroy(c->own_stream);
    delete c;
    return fail(KM_ERR_HIP, std::string("km_create: ") + hipGetErrorString(e));
  }
  *out = c;
  return KM_OK;
}

int km_destroy(km_ctx* c) {
  if (!c) return KM_OK;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  free_centroids(c);
  free_data(c);
  hfree(c->pinned);
  for (auto& e : c->staged)
    if (e) (void)hipEventDestroy(e);
  for (auto& v : c->ev)
    for (auto& p : v) {
      (void)hipEventDestroy(p.first);
      (void)hipEventDestroy(p.second);
    }
  for (auto e : c->pool) (void)hipEventDestroy(e);
  dfree(c->gate);
  free_repair(c);
  dfree(c->rep_sizes);
  dfree(c->rep_bases);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return KM_OK;
}

int km_set_stream(km_ctx* c, void* s) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  KM_HIP(hipSetDevice(c->device));
  {
    // a deferred assign runs on the stream it was enqueued for
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  KM_HIP(hipStreamSynchronize(c->stream));
  c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own_stream;
  return KM_OK;
}

int km_sync(km_ctx* c) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_info_get(km_ctx* c, km_info* out) {
  KM_REQUIRE(c && out, KM_ERR_ARG, "null arg");
  out->n = c->g.n;
  out->d = c->g.d;
  out->dp = c->g.dp;
  out->k = c->g.k;
  out->kp = c->g.kp;
  out->path = c->path;
  out->n_cu = c->n_cu;
  out->device = c->device;
  out->fused_stats = (c->path == 1) || c->fused;
  out->delta_stats = c->last_delta ? 1 : 0;
  return KM_OK;
}

int km_load_begin(km_ctx* c, int64_t n, int32_t d) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  KM_REQUIRE(n >= 0 && n < (int64_t)UINT32_MAX, KM_ERR_ARG, "km_load_begin: n out of range");
  KM_REQUIRE(d > 0, KM_ERR_ARG, "km_load_begin: d must be positive");
  KM_HIP(hipSetDevice(c->device));
  {
    // a deferred assign reads the rows being replaced (flush first)
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  KM_HIP(hipStreamSynchronize(c->stream));
  free_data(c);
  free_centroids(c);
  c->g = km::Geometry{};
  c->g.n = n;
  c->g.d = d;
  c->g.dp = choose_dp(d);
  const int64_t rows = std::max<int64_t>(n, 1);
  KM_HIP(hipMalloc(&c->X, sizeof(float) * rows * c->g.dp));
  KM_HIP(hipMemsetAsync(c->X, 0, sizeof(float) * rows * c->g.dp, c->stream));
  KM_HIP(hipMalloc(&c->labels, sizeof(int32_t) * rows));
  KM_HIP(hipMalloc(&c->queue, sizeof(km::QEntry) * km::queue_capacity(rows, c->n_cu)));
  KM_HIP(hipMalloc(&c->qcount, sizeof(uint32_t) * km::qcount_words(c->n_cu)));
  KM_HIP(hipMalloc(&c->small_ctr, sizeof(uint32_t) * 3));
  KM_HIP(hipMemsetAsync(c->small_ctr, 0, sizeof(uint32_t) * 3, c->stream));
  KM_HIP(hipMalloc(&c->moments, sizeof(double) * (d + 1)));
  KM_HIP(hipMalloc(&c->xabs, sizeof(float)));
  KM_HIP(hipMalloc(&c->xnorm, sizeof(float) * rows));
  KM_HIP(hipMemsetAsync(c->xabs, 0, sizeof(float), c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  c->loaded = true;
  return KM_OK;
}

int km_load_rows(km_ctx* c, int64_t row0, const float* rows, int64_t nrows) {
  KM_REQUIRE(c && c->loaded, KM_ERR_STATE, "km_load_rows: call km_load_begin first");
  KM_REQUIRE(row0 >= 0 && nrows >= 0 && row0 + nrows <= c->g.n, KM_ERR_ARG, "km_load_rows: rows out of range");
  if (nrows == 0) return KM_OK;
  KM_REQUIRE(rows, KM_ERR_ARG, "km_load_rows: null rows");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);  // it must read the rows it was called for
    if (rcf != KM_OK) return rcf;
  }
  c->delta_ready = false;  // the rows behind the labels change
  const int d = c->g.d, dp = c->g.dp;
  // double-buffered pinned staging: the host fills one half while the DMA
  // of the other is in flight (one event per half, one sync at the end)
  const size_t chunk_floats = (size_t)16 << 20;  // 2 x 64 MiB
  if (!c->pinned) {
    KM_HIP(hipHostMalloc(&c->pinned, 2 * chunk_floats * sizeof(float), hipHostMallocDefault));
    c->pinned_floats = chunk_floats;
    for (auto& e : c->staged) KM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  const int64_t per = std::max<int64_t>(1, (int64_t)(c->pinned_floats / d));
  KM_REQUIRE((size_t)d <= c->pinned_floats, KM_ERR_ARG, "km_load_rows: row wider than the staging buffer");
  int half = 0;
  bool used[2] = {false, false};
  for (int64_t r = 0; r < nrows; r += per, half ^= 1) {
    const int64_t m = std::min(per, nrows - r);
    float* buf = c->pinned + (size_t)half * c->pinned_floats;
    if (used[half]) KM_HIP(hipEventSynchronize(c->staged[half]));  // its previous copy is done
    memcpy(buf, rows + r * d, sizeof(float) * m * d);
    KM_HIP(hipMemcpy2DAsync(c->X + (row0 + r) * dp, sizeof(float) * dp, buf, sizeof(float) * d,
                            sizeof(float) * d, m, hipMemcpyHostToDevice, c->stream));
    KM_HIP(hipEventRecord(c->staged[half], c->stream));
    used[half] = true;
    KM_HIP(km::launch_absmax(c->X + (row0 + r) * dp, m * dp, c->xabs, c->stream));
    km::Geometry sub = c->g;
    sub.n = m;
    KM_HIP(km::launch_row_norm(c->X + (row0 + r) * dp, sub, c->xnorm + row0 + r, c->stream));
  }
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_generate_blobs(km_ctx* c, int64_t n, int32_t d, int64_t global_row0, int32_t n_centers, float box,
                      float stddev, uint64_t seed) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  KM_REQUIRE(n_centers > 0, KM_ERR_ARG, "n_centers must be positive");
  int rc = km_load_begin(c, n, d);
  if (rc != KM_OK) return rc;
  KM_HIP(km::launch_gen_blobs(c->X, c->g, global_row0, n_centers, box, stddev, seed, c->stream));
  KM_HIP(km::launch_absmax(c->X, c->g.n * c->g.dp, c->xabs, c->stream));
  KM_HIP(km::launch_row_norm(c->X, c->g, c->xnorm, c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_sum_x(km_ctx* c, double* out) {
  KM_REQUIRE(c && c->loaded && out, KM_ERR_STATE, "km_sum_x: no data");
  KM_HIP(hipSetDevice(c->device));
  KM_HIP(hipMemsetAsync(c->moments, 0, sizeof(double) * (c->g.d + 1), c->stream));
  KM_HIP(km::launch_sum_x(c->X, c->g, c->moments, c->stream));
  KM_HIP(hipMemcpyAsync(out, c->moments, sizeof(double) * c->g.d, hipMemcpyDeviceToHost, c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_set_screen(km_ctx* c, int32_t mode) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  KM_REQUIRE(mode >= -1 && mode <= KM_SCREEN_ONE, KM_ERR_ARG, "km_set_screen: mode must be -1..5");
#ifndef KM_DIAG
  // the fast screens (k_fused1) lost end to end on every BASELINE shape
  // (DESIGN.md "Fast screen"): built in the diagnostic library only
  KM_REQUIRE(mode <= km::KM_SCREEN_X3_REFINE || mode == KM_SCREEN_S1 || mode == KM_SCREEN_ONE, KM_ERR_UNSUPPORTED,
             "km_set_screen: fast screens (modes 2, 3) are in the diagnostic build only");
#endif
  c->screen_forced = mode;
  if (mode >= 0 && mode != KM_SCREEN_S1 && mode != KM_SCREEN_ONE) c->screen = mode;
  return KM_OK;
}

int km_get_screen(km_ctx* c, int32_t* mode) {
  KM_REQUIRE(c && mode, KM_ERR_ARG, "null ctx");
  // the screen of the next fused assign with statistics
  *mode = (use_s1(c, true) || (c->s1 && !c->fused && (c->screen_forced < 0 || c->screen_forced == KM_SCREEN_S1)))
              ? KM_SCREEN_S1
              : one_screen(c) ? KM_SCREEN_ONE : c->screen;
  return KM_OK;
}

int km_set_sse(km_ctx* c, int32_t enable) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  {
    const int rcf = flush_assign(c);  // launched with the residual choice it was called under
    if (rcf != KM_OK) return rcf;
  }
  c->want_sse = enable != 0;
  return KM_OK;
}

int km_set_centroids(km_ctx* c, const double* C, int32_t k, int32_t d) {
  KM_REQUIRE(c && c->loaded, KM_ERR_STATE, "km_set_centroids: load data first");
  KM_REQUIRE(C, KM_ERR_ARG, "km_set_centroids: null C");
  KM_REQUIRE(k > 0, KM_ERR_ARG, "km_set_centroids: k must be positive");
  KM_REQUIRE(d == c->g.d, KM_ERR_ARG,
             "km_set_centroids: d=" + std::to_string(d) + " != data d=" + std::to_string(c->g.d));
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  if (k != c->k_alloc) {
    KM_HIP(hipStreamSynchronize(c->stream));
    double* external = (c->stats && c->stats != c->stats_own) ? c->stats : nullptr;
    (void)external;
    free_centroids(c);
    c->g.k = k;
    c->g.kp = (k + 63) / 64 * 64;
    const int kp = c->g.kp, dp = c->g.dp;
    KM_HIP(hipMalloc(&c->C64_cur, sizeof(double) * k * d));
    KM_HIP(hipMalloc(&c->C64_new, sizeof(double) * k * d));
    KM_HIP(hipMalloc(&c->C64T, sizeof(double) * k * d));
    KM_HIP(hipMalloc(&c->C64P, sizeof(double) * kp * dp));
    KM_HIP(hipMalloc(&c->C32, sizeof(float) * kp * dp));
    KM_HIP(hipMalloc(&c->Chi, sizeof(_Float16) * kp * dp));
    KM_HIP(hipMalloc(&c->Clo, sizeof(_Float16) * kp * dp));
    KM_HIP(hipMalloc(&c->cn2, sizeof(float) * kp));
    KM_HIP(hipMalloc(&c->cn2s, sizeof(float) * kp));
    KM_HIP(hipMalloc(&c->ChiF, sizeof(_Float16) * kp * dp));
    KM_HIP(hipMalloc(&c->CloF, sizeof(_Float16) * kp * dp));
    KM_HIP(hipMalloc(&c->bnd, sizeof(float) * 16));
    c->bal = c->bnd + 4;  // [0, 1]: screening-bound constants; bal[0..10]: fast screen image maxima and bound constants
    KM_HIP(hipMalloc(&c->cmax, sizeof(float)));
    KM_HIP(hipMalloc(&c->cabs, sizeof(float)));
    KM_HIP(hipMalloc(&c->stats_own, sizeof(double) * stats_len(c->g)));
    KM_HIP(hipMalloc(&c->work, sizeof(double) * 3 * k));
    KM_HIP(hipMalloc(&c->counts_dev, sizeof(int64_t) * k));
    KM_HIP(hipMalloc(&c->status_dev, sizeof(km::DevStatus)));
    KM_HIP(hipHostMalloc(&c->status_host, sizeof(km::DevStatus), hipHostMallocDefault));
    KM_HIP(hipHostMalloc(&c->counts_host, sizeof(int64_t) * k, hipHostMallocDefault));
    KM_HIP(hipMalloc(&c->hist, sizeof(km::DevStatus) * KM_MAX_BATCH));
    KM_HIP(hipHostMalloc(&c->hist_host, sizeof(km::DevStatus) * KM_MAX_BATCH, hipHostMallocDefault));
    KM_HIP(hipMalloc(&c->hist_counts, sizeof(int64_t) * (size_t)k * KM_MAX_BATCH));
    KM_HIP(hipHostMalloc(&c->hist_counts_host, sizeof(int64_t) * (size_t)k * KM_MAX_BATCH, hipHostMallocDefault));
    c->stats = c->stats_own;
    c->stats_clean = false;
    c->k_alloc = k;
    if (km::small_path_ok(c->g))
      c->path = 1;
    else if (km::mfma_path_ok(c->g))
      c->path = 2;
    else
      c->path = 0;
    c->fused = (c->path == 2) && km::fused_path_ok(c->g) && !fused_disabled();
    // k_s1 beside the fused screen (c3 class: delta statistics) or in place
    // of the unfused screen (c4 class: labels, then the statistics pass)
    c->s1 = (c->path == 2) && (!c->fused || km::fused16_ok(c->g)) && km::s1_ok(c->g) &&
            km::diag_env("KM_S1", 1) != 0;
    c->mdelta_geo = (c->path == 2) && !c->fused && !c->s1 && c->g.dp % 32 == 0 && c->g.dp <= 128 &&
                    c->g.k <= 65535 && km::diag_env("KM_MDELTA", 1) != 0;
    if (c->mdelta_geo) KM_HIP(hipMalloc(&c->stats_full, sizeof(double) * stats_len(c->g)));
    if (c->s1) {
      const size_t nt = km::s1_table_entries(c->g);
      KM_HIP(hipMalloc(&c->s1_perm, sizeof(int32_t) * nt));
      KM_HIP(hipMalloc(&c->s1_cft, sizeof(float) * nt * (dp + 4)));
      KM_HIP(hipMalloc(&c->s1_cn2o, sizeof(float) * kp));
      KM_HIP(hipMalloc(&c->s1_img, sizeof(_Float16) * kp * dp));
      KM_HIP(hipMalloc(&c->s1_cst, sizeof(float) * 8));
      KM_HIP(hipMalloc(&c->stats_full, sizeof(double) * stats_len(c->g)));
      KM_HIP(hipMalloc(&c->chg, sizeof(uint2) * km::s1_chg_entries(c->g, c->n_cu)));
      KM_HIP(hipMalloc(&c->chg_cnt, sizeof(uint32_t) * km::s1_wave_slots(c->n_cu)));
    }
  }
  c->s1_recolor = true;
  c->s1_color_age = 0;
  c->s1_batches = 0;
  c->delta_ready = false;
  c->stats_pending = 0;
  KM_HIP(hipMemcpyAsync(c->C64_cur, C, sizeof(double) * k * d, hipMemcpyHostToDevice, c->stream));
  int rc = prep(c);
  if (rc != KM_OK) return rc;
  KM_HIP(hipStreamSynchronize(c->stream));
  c->have_c = true;
  c->screen = c->screen_forced >= 0 ? c->screen_forced : km::KM_SCREEN_X3_REFINE;
  c->fast_blocked = false;
  c->rep_armed = c->rep_enabled;
  return KM_OK;
}

int km_get_centroids(km_ctx* c, int32_t which, double* out) {
  KM_REQUIRE(c && c->have_c && out, KM_ERR_STATE, "km_get_centroids: no centroids");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  const double* src = which ? c->C64_new : c->C64_cur;
  KM_HIP(hipMemcpyAsync(out, src, sizeof(double) * c->g.k * c->g.d, hipMemcpyDeviceToHost, c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_assign_stats(km_ctx* c) {
  KM_REQUIRE(c && c->have_c, KM_ERR_STATE, "km_assign_stats: set centroids first");
  KM_REQUIRE(c->path != 0, KM_ERR_UNSUPPORTED,
             "km_assign_stats: no kernel for d=" + std::to_string(c->g.d) + " (supported: d <= 2048)");
  KM_HIP(hipSetDevice(c->device));
  int rc = flush_assign(c);
  if (rc != KM_OK) return rc;
  if (fold_ok(c)) {
    // launched by km_update_async together with the update
    if (c->prep_of != c->C64_cur) {
      rc = prep(c);
      if (rc != KM_OK) return rc;
    }
    c->assign_pending = true;
    return KM_OK;
  }
  return run_assign(c, true);
}

int km_stats_buffer(km_ctx* c, void** p, int64_t* len) {
  KM_REQUIRE(c && c->have_c && p && len, KM_ERR_STATE, "km_stats_buffer: set centroids first");
  {
    const int rc = flush_assign(c);
    if (rc != KM_OK) return rc;
  }
  c->stats_exported = true;
  *p = c->stats;
  *len = (int64_t)stats_len(c->g);
  return KM_OK;
}

int km_bind_stats_buffer(km_ctx* c, void* p) {
  KM_REQUIRE(c && c->have_c, KM_ERR_STATE, "km_bind_stats_buffer: set centroids first");
  {
    const int rc = flush_assign(c);
    if (rc != KM_OK) return rc;
  }
  c->stats = p ? reinterpret_cast<double*>(p) : c->stats_own;
  c->stats_clean = false;
  return KM_OK;
}

static int fast_mode() {
#ifdef KM_DIAG
  static const int m = km::diag_env("KM_FAST", 1);  // diagnostic build: 0 off, 1 / 2 row parts
  return m == 0 ? -1 : (m == 2 ? km::KM_SCREEN_FAST2 : km::KM_SCREEN_FAST1);
#else
  return -1;  // product build: no fast screen
#endif
}

static void note_queue(km_ctx* c, const km::DevStatus& s) {
  if (c->screen_forced >= 0) return;
  const int64_t q = (int64_t)s.q_rerank + s.q_full;
  const bool was_fast = c->screen >= km::KM_SCREEN_FAST1;
  if (was_fast && q * 128 > c->g.n) c->fast_blocked = true;
  if (was_fast && !c->fast_blocked) return;
  if (q * 64 > c->g.n && !was_fast)
    c->screen = km::KM_SCREEN_X3_REFINE;
  else if (!was_fast && q * 2048 < c->g.n && !c->fast_blocked && fast_mode() >= 0 && km::fast_path_ok(c->g))
    c->screen = fast_mode();
  else
    c->screen = km::KM_SCREEN_X3;
}

int km_update(km_ctx* c, km_status* st, int64_t* counts) {
  KM_REQUIRE(c && c->have_c, KM_ERR_STATE, "km_update: set centroids first");
  KM_REQUIRE(!c->in_batch, KM_ERR_STATE, "km_update: inside a batch (use km_update_async)");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  const double* src = nullptr;
  {
    const int rca = apply_stats(c, &src, !km::update_one_ok(c->g));
    if (rca != KM_OK) return rca;
  }
  {
    ProfScope ps(c, KM_K_UPDATE);
    KM_HIP(km::launch_update(const_cast<double*>(src), c->C64_cur, c->g, c->C64_new, c->work, c->counts_dev, c->qcount,
                             c->ql.nwaves, c->status_dev, c->gate, -1.0, 0, c->stream, 0, nullptr, nullptr,
                             take_sse_corr(c)));
  }
  KM_HIP(hipMemcpyAsync(c->status_host, c->status_dev, sizeof(km::DevStatus), hipMemcpyDeviceToHost, c->stream));
  KM_HIP(hipMemcpyAsync(c->counts_host, c->counts_dev, sizeof(int64_t) * c->g.k, hipMemcpyDeviceToHost, c->stream));
  {
    // images of the new centroids for the next iteration, queued behind the
    // status copies (used after km_commit unless km_replace_rows changes them)
    const int rc = prep(c, c->C64_new);
    if (rc != KM_OK) return rc;
  }
  KM_HIP(hipStreamSynchronize(c->stream));
  const km::DevStatus& s = *c->status_host;
  note_queue(c, s);
  if (st) {
    st->sse = s.sse;
    st->max_shift = s.max_shift;
    st->n_empty = s.n_empty;
    st->nonfinite = s.nonfinite;
    st->q_rerank = s.q_rerank;
    st->q_full = s.q_full;
    st->ran = s.ran;
    st->stop_reason = s.stop;
    st->repaired = 0;
  }
  if (counts) memcpy(counts, c->counts_host, sizeof(int64_t) * c->g.k);
  return s.n_empty > 0 ? KM_EMPTY : KM_OK;
}

int km_set_layout(km_ctx* c, const int64_t* sizes, int32_t nparts, int64_t row0, int32_t device_repair) {
  KM_REQUIRE(c && c->loaded, KM_ERR_STATE, "km_set_layout: load data first");
  KM_REQUIRE(nparts >= 0 && (nparts == 0 || sizes), KM_ERR_ARG, "km_set_layout: bad partitions");
  KM_HIP(hipSetDevice(c->device));
  {
    // a deferred assign was decided under the old repair arming (fold_ok)
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  KM_HIP(hipStreamSynchronize(c->stream));
  free_repair(c);
  dfree(c->rep_sizes);
  dfree(c->rep_bases);
  c->rep_enabled = false;
  c->rep_nparts = nparts;
  c->rep_total = 0;
  c->rep_maxpart = 0;
  c->rep_row0 = row0;
  std::vector<int64_t> bases(nparts);
  for (int i = 0; i < nparts; ++i) {
    KM_REQUIRE(sizes[i] >= 0, KM_ERR_ARG, "km_set_layout: negative partition size");
    bases[i] = c->rep_total;
    c->rep_total += sizes[i];
    c->rep_maxpart = std::max(c->rep_maxpart, sizes[i]);
  }
  KM_REQUIRE(device_repair >= 0 && device_repair <= 2, KM_ERR_ARG, "km_set_layout: device_repair must be 0, 1 or 2");
  c->rep_mode = device_repair;
  if (device_repair) {
    // mode 1: every replacement row is resident here (one rank holding all
    // rows); mode 2: this context holds rows [row0, row0 + n) of the dataset
    KM_REQUIRE(device_repair == 2 || (row0 == 0 && c->rep_total == c->g.n), KM_ERR_ARG,
               "km_set_layout: device repair mode 1 needs every row of the dataset on this context");
    KM_REQUIRE(nparts > 0 && row0 >= 0 && row0 + c->g.n <= c->rep_total, KM_ERR_ARG,
               "km_set_layout: this context's rows lie outside the layout");
    KM_HIP(hipMalloc(&c->rep_sizes, sizeof(int64_t) * nparts));
    KM_HIP(hipMalloc(&c->rep_bases, sizeof(int64_t) * nparts));
    KM_HIP(hipMemcpy(c->rep_sizes, sizes, sizeof(int64_t) * nparts, hipMemcpyHostToDevice));
    KM_HIP(hipMemcpy(c->rep_bases, bases.data(), sizeof(int64_t) * nparts, hipMemcpyHostToDevice));
    c->rep_enabled = true;
  }
  c->rep_armed = c->rep_enabled;
  return KM_OK;
}

int km_batch_begin(km_ctx* c) {
  KM_REQUIRE(c && c->have_c, KM_ERR_STATE, "km_batch_begin: set centroids first");
  KM_REQUIRE(!c->in_batch, KM_ERR_STATE, "km_batch_begin: a batch is open");
  KM_HIP(hipSetDevice(c->device));
  KM_HIP(hipMemsetAsync(c->gate, 0, sizeof(int), c->stream));
  if (c->s1 && (++c->s1_batches <= 3 || ++c->s1_color_age >= 4)) {
    // the chain colouring follows the centroids at each of the first three
    // batches after new centroids (4 + 8 + 16 iterations, while they move
    // most), then every fourth batch (batches grow to 32 iterations; one
    // colouring is a sequential pass over k, ~0.8 ms at k = 256).  A stale
    // colouring can only queue rows, never mislabel them (the certificate
    // holds for any colouring: km_screen1.hip k_s1_color)
    c->s1_recolor = true;
    c->s1_color_age = 0;
    if (c->prep_of == c->C64_cur) c->prep_of = nullptr;
  }
  c->in_batch = true;
  c->batch_n = 0;
  ++c->batch_seq;
  return KM_OK;
}

static int finish_update(km_ctx* c, int slot, bool fold_prep);

int km_update_async(km_ctx* c, double tol, int64_t empty_seed) {
  KM_REQUIRE(c && c->have_c && c->in_batch, KM_ERR_STATE, "km_update_async: call km_batch_begin first");
  KM_REQUIRE(!c->rep_wait, KM_ERR_STATE, "km_update_async: the last iteration's km_repair_apply_async is missing");
  KM_REQUIRE(c->batch_n < KM_MAX_BATCH, KM_ERR_ARG, "km_update_async: more than KM_MAX_BATCH iterations in a batch");
  KM_REQUIRE(tol >= 0.0, KM_ERR_ARG, "km_update_async: tolerance must be >= 0");
  KM_HIP(hipSetDevice(c->device));
  const int slot = c->batch_n;
  const bool repair = c->rep_enabled && c->rep_armed;
  // one-workgroup update: clears the statistics and, on the small path with
  // no repair behind it, writes the next assign's centroid images itself
  const bool one = km::update_one_ok(c->g);
  const bool fold_prep = one && c->path == 1 && !repair;
  if (c->assign_pending && !fold_ok(c)) {
    // the fold was decided at km_assign_stats; if its conditions no longer
    // hold (a stats buffer bound or exported since, the repair re-armed),
    // the assign runs on its own and the update below is the usual launch
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  if (c->assign_pending) {
    // one launch: assign + sums + queued rows + update (last workgroup)
    c->assign_pending = false;
    c->ql = km::QLayout{0, 0};
    if (!c->stats_clean) KM_HIP(hipMemsetAsync(c->stats, 0, sizeof(double) * stats_len(c->g), c->stream));
    km::SmallTail t = small_tail(c);
    t.fold = 1;
    t.old = c->C64_cur;
    t.out = c->C64_new;
    t.counts = c->hist_counts + (size_t)slot * c->g.k;
    t.st = c->hist + slot;
    t.gate = c->gate;
    t.stop_tol = tol;
    t.dev_repair = 0;
    t.C32n = fold_prep ? c->C32 : nullptr;
    t.cmaxn = fold_prep ? c->cmax : nullptr;
    {
      ProfScope ps(c, KM_K_ASSIGN, true);
      KM_HIP(km::launch_assign_small(c->X, c->g, c->C32, c->C64_cur, c->cmax, c->labels, c->stats, 1,
                                     c->want_sse ? 1 : 0, c->n_cu, c->gate, c->stream, t));
    }
    c->stats_clean = true;  // the update cleared them
    return finish_update(c, slot, fold_prep);
  }
  const double* src = nullptr;
  {
    // (k_update_one clears its input: it reads the folded sums in stats)
    const int rca = apply_stats(c, &src, !one);
    if (rca != KM_OK) return rca;
  }
  {
    ProfScope ps(c, KM_K_UPDATE);
    KM_HIP(km::launch_update(one ? c->stats : const_cast<double*>(src), c->C64_cur, c->g, c->C64_new, c->work,
                             c->hist_counts + (size_t)slot * c->g.k, c->qcount, c->ql.nwaves, c->hist + slot,
                             c->gate, tol, repair ? 1 : 0, c->stream, one ? 1 : 0, fold_prep ? c->C32 : nullptr,
                             fold_prep ? c->cmax : nullptr, take_sse_corr(c)));
  }
  if (one) c->stats_clean = true;
  if (repair) {
    KM_REQUIRE(empty_seed >= 0, KM_ERR_ARG, "km_update_async: negative empty-cluster seed");
    const int rc = ensure_repair(c);
    if (rc != KM_OK) return rc;
    if (c->rep_mode == 2) {
      // rows spread over ranks: the caller all-reduces km_repair_buffer, then
      // km_repair_apply_async finishes this iteration
      KM_HIP(km::launch_repair_pick(c->gate, c->hist_counts + (size_t)slot * c->g.k, c->g, c->rep_total,
                                    -std::log(0.00005), (uint64_t)empty_seed, c->rep_empty, c->rep_pcounts,
                                    c->rep_picks, c->rep_samples, c->rep_cp, c->rep_sizes, c->rep_bases,
                                    c->rep_nparts, c->X, c->rep_row0, c->hist + slot, c->rep_rows, c->rep_pending,
                                    c->stream));
      c->rep_wait = true;
      c->rep_tol = tol;
      c->rep_fold = fold_prep;
      return KM_OK;
    }
    KM_HIP(km::launch_repair(c->gate, c->hist_counts + (size_t)slot * c->g.k, c->g, c->rep_total,
                             -std::log(0.00005), (uint64_t)empty_seed, c->rep_empty, c->rep_pcounts, c->rep_picks,
                             c->rep_samples, c->rep_cp, c->rep_sizes, c->rep_bases, c->rep_nparts, c->X,
                             c->rep_row0, c->C64_cur, c->C64_new, c->hist + slot, tol, c->stream));
  }
  return finish_update(c, slot, fold_prep);
}

// the tail of an iteration enqueued in a batch: slot bookkeeping and the
// speculative commit of the new centroids
static int finish_update(km_ctx* c, int slot, bool fold_prep) {
  c->slot_cur[slot] = c->C64_cur;
  c->slot_new[slot] = c->C64_new;
  // speculative commit (kmeans_spark.py:307): the next iteration reads the
  // new centroids; a stopped batch's later kernels (prep included) no-op and
  // km_batch_end restores the state after the last iteration that ran
  if (fold_prep) {
    c->prep_of = c->C64_new;  // written by the update (it ran whenever the next assign runs)
  } else {
    const int rc = prep(c, c->C64_new);
    if (rc != KM_OK) return rc;
  }
  std::swap(c->C64_cur, c->C64_new);
  c->batch_n = slot + 1;
  return KM_OK;
}

int km_repair_state(km_ctx* c, int32_t* armed, int32_t* waiting) {
  KM_REQUIRE(c && armed && waiting, KM_ERR_ARG, "km_repair_state: null argument");
  *armed = (c->rep_enabled && c->rep_armed) ? 1 : 0;
  *waiting = c->rep_wait ? 1 : 0;
  return KM_OK;
}

int km_repair_buffer(km_ctx* c, void** p, int64_t* len) {
  KM_REQUIRE(c && p && len, KM_ERR_ARG, "km_repair_buffer: null argument");
  KM_REQUIRE(c->rep_mode == 2 && c->have_c, KM_ERR_STATE, "km_repair_buffer: needs km_set_layout mode 2 and centroids");
  if (!c->rep_rows) {
    const int rc = ensure_repair(c);
    if (rc != KM_OK) return rc;
  }
  *p = c->rep_rows;
  *len = (int64_t)c->g.k * c->g.d;
  return KM_OK;
}

int km_bind_repair_buffer(km_ctx* c, void* p) {
  KM_REQUIRE(c && c->rep_mode == 2 && c->have_c, KM_ERR_STATE,
             "km_bind_repair_buffer: needs km_set_layout mode 2 and centroids");
  const int rc = ensure_repair(c);
  if (rc != KM_OK) return rc;
  c->rep_rows = p ? reinterpret_cast<double*>(p) : c->rep_rows_own;
  return KM_OK;
}

int km_repair_apply_async(km_ctx* c) {
  KM_REQUIRE(c && c->in_batch && c->rep_wait, KM_ERR_STATE,
             "km_repair_apply_async: no repair pick pending (km_update_async in layout mode 2)");
  KM_HIP(hipSetDevice(c->device));
  const int slot = c->batch_n;
  KM_HIP(km::launch_repair_apply(c->gate, c->g, c->rep_empty, c->C64_cur, c->C64_new, c->hist + slot, c->rep_tol,
                                 c->rep_rows, c->rep_pending, c->stream));
  c->rep_wait = false;
  return finish_update(c, slot, c->rep_fold);
}

int km_batch_end(km_ctx* c, km_status* st, int64_t* counts, int32_t* n_ran) {
  KM_REQUIRE(c && c->in_batch, KM_ERR_STATE, "km_batch_end: no open batch");
  KM_REQUIRE(n_ran, KM_ERR_ARG, "km_batch_end: null n_ran");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  const int m = c->batch_n;
  if (m > 0) {
    KM_HIP(hipMemcpyAsync(c->hist_host, c->hist, sizeof(km::DevStatus) * m, hipMemcpyDeviceToHost, c->stream));
    KM_HIP(hipMemcpyAsync(c->hist_counts_host, c->hist_counts, sizeof(int64_t) * (size_t)c->g.k * m,
                          hipMemcpyDeviceToHost, c->stream));
  }
  KM_HIP(hipMemsetAsync(c->gate, 0, sizeof(int), c->stream));  // later launches run again
  KM_HIP(hipStreamSynchronize(c->stream));
  c->in_batch = false;
  c->batch_n = 0;
  c->rep_wait = false;  // an iteration left without its km_repair_apply_async did not run
  int ran = 0;
  while (ran < m && c->hist_host[ran].ran) ++ran;
  *n_ran = ran;
  for (auto& v : c->ev) {
    size_t w = 0;
    for (size_t i = 0; i < v.size(); ++i) {
      if (v[i].batch == c->batch_seq && v[i].slot >= ran) {  // a no-op launch of the stopped batch
        c->pool.push_back(v[i].first);
        c->pool.push_back(v[i].second);
      } else {
        v[w++] = v[i];
      }
    }
    v.resize(w);
  }
  if (ran > 0) {
    // the state after the last iteration that ran, before its commit (as
    // after km_update): its old / new buffers, the new one's images prepared
    c->C64_cur = c->slot_cur[ran - 1];
    c->C64_new = c->slot_new[ran - 1];
    // the iteration that raised the gate had its own prep gated too
    c->prep_of = c->hist_host[ran - 1].stop ? nullptr : c->C64_new;
    note_queue(c, c->hist_host[ran - 1]);
    if (c->rep_enabled) {
      bool any_empty = false;
      for (int i = 0; i < ran; ++i) any_empty |= c->hist_host[i].n_empty > 0;
      // an empty stop (disarmed) re-arms; a batch without empties disarms
      c->rep_armed = any_empty;
    }
  } else if (m > 0) {
    c->C64_cur = c->slot_cur[0];
    c->C64_new = c->slot_new[0];
    c->prep_of = nullptr;
  }
  for (int i = 0; i < ran; ++i) {
    const km::DevStatus& s = c->hist_host[i];
    if (st) {
      st[i].sse = s.sse;
      st[i].max_shift = s.max_shift;
      st[i].n_empty = s.n_empty;
      st[i].nonfinite = s.nonfinite;
      st[i].q_rerank = s.q_rerank;
      st[i].q_full = s.q_full;
      st[i].ran = s.ran;
      st[i].stop_reason = s.stop;
      st[i].repaired = s.repaired;
    }
    if (counts) memcpy(counts + (size_t)i * c->g.k, c->hist_counts_host + (size_t)i * c->g.k, sizeof(int64_t) * c->g.k);
  }
  return KM_OK;
}

int km_replace_rows(km_ctx* c, const int32_t* ids, const double* rows, int32_t n) {
  KM_REQUIRE(c && c->have_c, KM_ERR_STATE, "km_replace_rows: set centroids first");
  KM_REQUIRE(n >= 0 && (n == 0 || (ids && rows)), KM_ERR_ARG, "km_replace_rows: bad args");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  if (n == 0) return KM_OK;
  if (c->prep_of == c->C64_new) c->prep_of = nullptr;  // its images are stale now
  c->screen = c->screen_forced >= 0 ? c->screen_forced : km::KM_SCREEN_X3_REFINE;
  c->fast_blocked = false;
  c->rep_armed = c->rep_enabled;
  std::vector<int64_t> ids64(n);
  for (int i = 0; i < n; ++i) {
    KM_REQUIRE(ids[i] >= 0 && ids[i] < c->g.k, KM_ERR_ARG, "km_replace_rows: cluster id out of range");
    ids64[i] = ids[i];
  }
  const int rc = ensure_scratch(c, n);
  if (rc != KM_OK) return rc;
  // one copy of the ids and rows, one scatter launch
  KM_HIP(hipMemcpyAsync(c->idx_scratch, ids64.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream));
  KM_HIP(hipMemcpyAsync(c->rows_scratch, rows, sizeof(double) * (size_t)n * c->g.d, hipMemcpyHostToDevice,
                        c->stream));
  KM_HIP(km::launch_scatter_rows(c->idx_scratch, c->rows_scratch, n, c->g.d, c->C64_new, c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_commit(km_ctx* c) {
  KM_REQUIRE(c && c->have_c, KM_ERR_STATE, "km_commit: set centroids first");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  std::swap(c->C64_cur, c->C64_new);
  return c->prep_of == c->C64_cur ? KM_OK : prep(c);
}

int km_gather_rows(km_ctx* c, const int64_t* idx, int32_t n, double* out) {
  KM_REQUIRE(c && c->loaded, KM_ERR_STATE, "km_gather_rows: no data");
  if (n <= 0) return KM_OK;
  KM_REQUIRE(idx && out, KM_ERR_ARG, "km_gather_rows: null arg");
  for (int i = 0; i < n; ++i)
    KM_REQUIRE(idx[i] >= 0 && idx[i] < c->g.n, KM_ERR_ARG, "km_gather_rows: index out of range");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  int rc = ensure_scratch(c, n);
  if (rc != KM_OK) return rc;
  KM_HIP(hipMemcpyAsync(c->idx_scratch, idx, sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream));
  KM_HIP(km::launch_gather_rows(c->X, c->g, c->idx_scratch, n, c->rows_scratch, c->stream));
  KM_HIP(hipMemcpyAsync(out, c->rows_scratch, sizeof(double) * n * c->g.d, hipMemcpyDeviceToHost, c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_bernoulli_sample(km_ctx* c, const uint64_t* seeds, const int64_t* sizes, const int64_t* bases, int32_t nparts,
                        double fraction, int64_t* out, int64_t cap, int64_t* n_out) {
  KM_REQUIRE(c && n_out, KM_ERR_ARG, "km_bernoulli_sample: null arg");
  *n_out = 0;
  if (nparts <= 0) return KM_OK;
  KM_REQUIRE(seeds && sizes && bases && (cap == 0 || out), KM_ERR_ARG, "km_bernoulli_sample: null arg");
  int64_t maxs = 0;
  for (int i = 0; i < nparts; ++i) {
    KM_REQUIRE(sizes[i] >= 0, KM_ERR_ARG, "km_bernoulli_sample: negative partition size");
    maxs = std::max(maxs, sizes[i]);
  }
  KM_REQUIRE(fraction >= 0.0 && fraction <= 1.0, KM_ERR_ARG, "km_bernoulli_sample: fraction out of [0, 1]");
  // per-partition slots: 4x the expected picks + 64 (more -> KM_ERR_ARG, the
  // caller falls back to its host sampler)
  const double expect = fraction * (double)maxs;
  KM_REQUIRE(expect * 4.0 + 64.0 < (double)(1 << 24), KM_ERR_ARG, "km_bernoulli_sample: sample too large for the device pass");
  const int cp = (int)(expect * 4.0) + 64;
  KM_HIP(hipSetDevice(c->device));
  const size_t bytes_in = (sizeof(uint64_t) + 2 * sizeof(int64_t)) * (size_t)nparts;
  const size_t bytes_out = sizeof(int64_t) * (size_t)nparts * cp + sizeof(int32_t) * (size_t)nparts;
  char* dbuf = nullptr;
  KM_HIP(hipMalloc(&dbuf, bytes_in + bytes_out));
  uint64_t* dseeds = reinterpret_cast<uint64_t*>(dbuf);
  int64_t* dsizes = reinterpret_cast<int64_t*>(dseeds + nparts);
  int64_t* dbases = dsizes + nparts;
  int64_t* dout = dbases + nparts;
  int32_t* dcounts = reinterpret_cast<int32_t*>(dout + (size_t)nparts * cp);
  std::vector<int64_t> hout((size_t)nparts * cp);
  std::vector<int32_t> hcounts(nparts);
  hipError_t e = hipMemcpyAsync(dseeds, seeds, sizeof(uint64_t) * nparts, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dsizes, sizes, sizeof(int64_t) * nparts, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(dbases, bases, sizeof(int64_t) * nparts, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = km::launch_bernoulli(dseeds, dsizes, dbases, nparts, fraction, dout, cp, dcounts, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(hcounts.data(), dcounts, sizeof(int32_t) * nparts, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess)
    e = hipMemcpyAsync(hout.data(), dout, sizeof(int64_t) * (size_t)nparts * cp, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(dbuf);
  if (e != hipSuccess) return fail(KM_ERR_HIP, std::string("km_bernoulli_sample: ") + hipGetErrorString(e));
  int64_t total = 0;
  for (int i = 0; i < nparts; ++i) {
    KM_REQUIRE(hcounts[i] <= cp, KM_ERR_ARG, "km_bernoulli_sample: more picks than the device pass holds");
    total += hcounts[i];
  }
  KM_REQUIRE(total <= cap, KM_ERR_ARG, "km_bernoulli_sample: output capacity too small");
  int64_t o = 0;
  for (int i = 0; i < nparts; ++i)
    for (int j = 0; j < hcounts[i]; ++j) out[o++] = hout[(size_t)i * cp + j];
  *n_out = total;
  return KM_OK;
}

int km_predict(km_ctx* c, int32_t* labels_out) {
  KM_REQUIRE(c && c->have_c, KM_ERR_STATE, "km_predict: set centroids first");
  KM_REQUIRE(c->path != 0, KM_ERR_UNSUPPORTED, "km_predict: unsupported geometry");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  int rc = run_assign(c, false);
  if (rc != KM_OK) return rc;
  c->delta_ready = false;  // the labels are now predict's, not the sums' assignment
  if (labels_out && c->g.n > 0)
    KM_HIP(hipMemcpyAsync(labels_out, c->labels, sizeof(int32_t) * c->g.n, hipMemcpyDeviceToHost, c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_labels(km_ctx* c, int32_t* labels_out) {
  KM_REQUIRE(c && c->loaded && labels_out, KM_ERR_STATE, "km_labels: no data");
  KM_HIP(hipSetDevice(c->device));
  {
    const int rcf = flush_assign(c);
    if (rcf != KM_OK) return rcf;
  }
  if (c->g.n > 0)
    KM_HIP(hipMemcpyAsync(labels_out, c->labels, sizeof(int32_t) * c->g.n, hipMemcpyDeviceToHost, c->stream));
  KM_HIP(hipStreamSynchronize(c->stream));
  return KM_OK;
}

int km_profile(km_ctx* c, int32_t enable) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  c->prof = enable;  // bitmask of (1 << KM_K_*); -1 = every phase
  return KM_OK;
}

int km_profile_every(km_ctx* c, int32_t period) {
  KM_REQUIRE(c, KM_ERR_ARG, "null ctx");
  KM_REQUIRE(period >= 1, KM_ERR_ARG, "km_profile_every: period must be >= 1");
  c->prof_period = period;
  for (auto& t : c->prof_tick) t = 0;
  return KM_OK;
}

int km_prof_read(km_ctx* c, int32_t kind, double* total_ms, int64_t* launches) {
  KM_REQUIRE(c && kind >= 0 && kind < KM_K_COUNT, KM_ERR_ARG, "km_prof_read: bad kind");
  KM_HIP(hipSetDevice(c->device));
  KM_HIP(hipStreamSynchronize(c->stream));
  double tot = 0.0;
  for (auto& p : c->ev[kind]) {
    float ms = 0.0f;
    KM_HIP(hipEventElapsedTime(&ms, p.first, p.second));
    tot += ms;
    c->pool.push_back(p.first);
    c->pool.push_back(p.second);
  }
  if (total_ms) *total_ms = tot;
  if (launches) *launches = (int64_t)c->ev[kind].size();
  c->ev[kind].clear();
  return KM_OK;
}

}  // extern "C"
