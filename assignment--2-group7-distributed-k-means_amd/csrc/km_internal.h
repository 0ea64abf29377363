// Internal declarations shared by km_kernels.hip (device code + launchers)
// and km_runtime.hip (context, memory, C-ABI).  Not part of the public ABI
// (that is include/kmeans_amd.h).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kmeans_amd.h"

namespace km {

// Timing of a phase's dominant kernel (bench, km_profile): the events ride in
// the kernel's own dispatch (hipExtLaunchKernelGGL) instead of two extra
// packets on the stream (~8 us of stream time per step at c2).  A ProfScope
// arms them; the next KM_TIMED_LAUNCH consumes them.
struct LaunchTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local LaunchTiming g_timing;
#define KM_TIMED_LAUNCH(KERNEL, GRID, BLOCK, LDS, STREAM, ...)                                               \
  do {                                                                                                     \
    if (::km::g_timing.start) {                                                                            \
      hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, STREAM, ::km::g_timing.start, ::km::g_timing.stop, 0, \
                            __VA_ARGS__);                                                                  \
      ::km::g_timing = ::km::LaunchTiming{};                                                               \
    } else {                                                                                               \
      hipLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, STREAM, __VA_ARGS__);                                    \
    }                                                                                                      \
  } while (0)

// Ambiguous-point queue entry written by the screening kernels and consumed
// by k_resolve (exact float64 re-rank of the reference's np.argmin).
struct QEntry {
  uint32_t row;   // local row
  uint32_t i1;    // best screened centroid
  uint32_t i2;    // second best screened centroid (kind 4: record of the candidate pool)
  uint32_t kind;  // 1 = re-rank {i1,i2}, 2 = full exact scan, 3 = scan of the chain j & 7 == i1 & 7,
                  // 4 = re-rank of a candidate list (k_assign_mfma)
};

// Per-iteration status produced on device by k_finalize (kmeans_spark.py:176-313
// quantities), copied to pinned host memory by km_update.
struct DevStatus {
  double sse;          // SSE of the assignment w.r.t. the pre-update centroids (L224-237)
  double max_shift;    // max_c ||new_c - old_c||  (L293-294), empties kept at old
  int32_t n_empty;     // clusters with no points (L186-188)
  int32_t nonfinite;   // any non-finite new centroid (L289)
  int32_t q_rerank;    // screened points re-ranked exactly
  int32_t q_full;      // screened points that needed the full exact scan
  int32_t ran;         // 0: the iteration was a no-op of a stopped batch
  int32_t stop;        // KM_STOP_* raised by this iteration (batches)
  int32_t repaired;    // empty clusters were replaced on the device (max_shift includes them)
  int32_t pad;
};
static_assert(sizeof(DevStatus) == 48, "layout of km_status");


// Per-wave segments of the ambiguous-point queue written by k_assign_mfma:
// wave w owns entries [w*seg, w*seg + qcount[2w]); qcount[2w+1] = full scans.
struct QLayout {
  uint32_t seg;
  uint32_t nwaves;
};

struct Geometry {
  int64_t n;    // local rows
  int32_t d;    // features
  int32_t dp;   // padded row stride of X (floats), multiple of 16
  int32_t k;    // clusters
  int32_t kp;   // padded cluster count (multiple of 64)
};

// ---- launchers (km_kernels.hip) -------------------------------------------
// C64P: float64 centroids padded to [kp][dp] (zero padding), the source of
// the SSE residuals (aligned rows, no per-feature bound checks)
hipError_t launch_prep_centroids(const double* C64, const Geometry& g, float* C32, float* cn2, float* cmax,
                                 float* cabs, double* C64T, double* C64P, const int* gate, hipStream_t s);
// fp16 hi/lo split of -2*c*s and ||c||^2 s^2 for the MFMA screen (s from the
// data and centroid abs maxima)
// the small path's images only (fp32 copy + max norm), one launch
hipError_t launch_prep_small(const double* C64, const Geometry& g, float* C32, float* cmax, const int* gate,
                             hipStream_t s);
hipError_t launch_prep_split(const float* C32, const Geometry& g, const float* cn2, const float* xabs,
                             const float* cabs, _Float16* Chi, _Float16* Clo, float* cn2s, const int* gate, hipStream_t s);
hipError_t launch_absmax(const float* X, int64_t nfloats, float* out, hipStream_t s);
// Small k*d path: direct-form fp32 screening (ambiguous rows queued, see below),
// optional fused statistics (LDS float64 table, replicated per lane).
// want_sse: also add every point's float64 residual ||x - c_label||^2 to
// stats[k (d+1)] (the SSE slot, kmeans_spark.py:224-237)
// The rows the fp32 bound cannot settle are queued; the last workgroup of the
// launch resolves them in float64 (and adds their sums) and, with fold, runs
// the one-workgroup update as well (an iteration in one launch).
struct SmallTail {
  uint32_t* queue;  // ambiguous rows (capacity n)
  uint32_t* qctr;   // queue length; zeroed again by the last workgroup
  uint32_t* done;   // [0] workgroups finished, [1] queued rows; zeroed again by the last workgroup
  int fold;         // run the one-workgroup update in the last workgroup
  const double* old;
  double* out;
  int64_t* counts;
  DevStatus* st;
  int* gate;
  double stop_tol;
  int dev_repair;
  float* C32n;  // the next iteration's images (prep folded in), or nullptr
  float* cmaxn;
  int kp;
  uint32_t* qout = nullptr;  // no fold: the queued-row count for the update's status (qcount[0..1])
  int rev = 0;  // sweep the rows from the last one down (alternate launches: the Infinity Cache holds the previous sweep's tail)
};
hipError_t launch_assign_small(const float* X, const Geometry& g, const float* C32, const double* C64,
                               const float* cmax, int32_t* labels, double* stats, int fuse_stats, int want_sse,
                               int n_cu, const int* gate, hipStream_t s, const SmallTail& tail);
bool small_path_ok(const Geometry& g);
// MFMA path: fp16x3 screening on v_mfma_f32_32x32x16_f16, top-3 keys,
// ambiguous points queued for the exact resolvers.
// cand / cand_ctr / cand_cap: pool of candidate lists (kind-4 queue entries,
// cand_rec_words() words each; the counter is zeroed by the launch); nullptr:
// every kind-2 point is left to the full scan
hipError_t launch_assign_mfma(const float* X, const Geometry& g, const _Float16* Chi, const _Float16* Clo,
                              const float* cn2s, const float* cmax, const float* xabs, const float* cabs,
                              int32_t* labels, QEntry* queue, uint32_t* qcount, int n_cu, QLayout* ql,
                              const int* gate, hipStream_t s, uint32_t* cand = nullptr, uint32_t* cand_ctr = nullptr,
                              uint32_t cand_cap = 0, int one = 0,
                              const float* C32 = nullptr, uint2* chg = nullptr, uint32_t* chg_cnt = nullptr);
int cand_rec_words();
// queue capacity (entries) and per-wave counter words needed for n rows
size_t queue_capacity(int64_t n, int n_cu);
size_t qcount_words(int n_cu);
bool mfma_path_ok(const Geometry& g);
// stats != nullptr: also add the resolved points' rows to the partial sums
// delta: the queued rows still hold their previous labels (delta statistics);
// each resolved row writes {row, old << 16 | new} into the change list chg of
// the screen, behind the screen's chg_cnt[w] entries of its wave segment w
// (re-rank entries first, then full scans: chg_cnt[w] + qcount[2w] +
// qcount[2w+1] <= seg entries), stats unused; launch_chg_delta folds them
// C32, cmax (the fp32 images and their largest norm): the full scans run an
// fp32 prefilter first and evaluate only the centroids it keeps in float64
hipError_t launch_resolve(const float* X, const Geometry& g, const double* C64, const double* C64T,
                          const QEntry* queue, const uint32_t* qcount, const QLayout& ql, int32_t* labels,
                          double* stats, int n_cu, const int* gate, hipStream_t s, double* sse = nullptr,
                          const uint32_t* cand = nullptr, uint32_t cand_cap = 0, int delta = 0,
                          const float* sse_c32 = nullptr, uint2* chg = nullptr, const uint32_t* chg_cnt = nullptr,
                          const float* C32 = nullptr, const float* cmax = nullptr);
// Fused assign + partial sums (kp*dp <= 16384 class): fp16 hi image in VGPRs,
// lo image + float64 sum table in LDS; decided points summed here, queued
// points (and their counts) by launch_resolve(stats).
bool fused_path_ok(const Geometry& g);
#ifdef KM_DIAG
#endif
// Tuning / ablation knob `name`: read from the environment only in the
// diagnostic build (make diag, -DKM_DIAG); the product library always uses
// `dflt`, so kernel selection depends on the geometry alone (and, for the
// per-key refinement in k_fused, on the last queue fraction: a cost choice
// with no effect on results, which are exact either way).
int diag_env(const char* name, int dflt);
// Screen of the fused kernel: fp16x3 with the global bound (X3), plus the
// per-key refinement (X3_REFINE), or the fast screen k_fused1 (one fp16 image,
// pairwise bound) with the row as one fp16 part (FAST1) or hi + lo (FAST2).
// Results are exact in every mode; the choice is a cost choice.
// (mode 4, KM_SCREEN_S1 of kmeans_amd.h: the one-MFMA screen with in-kernel
// re-scoring and delta statistics, km_screen1.hip; forcing 0 / 1 keeps
// k_fused16 on every assign)
enum { KM_SCREEN_X3 = 0, KM_SCREEN_X3_REFINE = 1, KM_SCREEN_FAST1 = 2, KM_SCREEN_FAST2 = 3 };
bool fast_path_ok(const Geometry& g);
// C32, cmax: fp32 centroids and max norm (fast screen image); bal: 2 floats of
// scratch (fast screen image error maxima)
hipError_t launch_fused(const float* X, const float* xnorm, const Geometry& g, const _Float16* Chi,
                        const _Float16* Clo, uint4* ChiF, uint4* CloF, const float* cn2s, const float* bnd,
                        const float* xabs, const float* cabs, int32_t* labels, QEntry* queue, uint32_t* qcount,
                        double* stats, int with_stats, int mode, int n_cu, QLayout* ql, const int* gate,
                        hipStream_t s, const float* C32, const float* cmax, float* bal, const double* C64P,
                        double* sse);
// bound constants of the fused screen (the MFMA shape it runs on: fused16_ok)
hipError_t launch_bound_consts(const float* cmax, const float* xabs, const float* cabs, const Geometry& g, float* bnd,
                               const int* gate, hipStream_t s);
// the fused screen runs on v_mfma_f32_16x16x32_f16 (k_fused16) for this geometry
bool fused16_ok(const Geometry& g);
hipError_t launch_row_norm(const float* X, const Geometry& g, float* xnorm, hipStream_t s);
// large k: counting sort of the labels + per-cluster float64 row sums (X read
// once); scratch = sorted_stats_words(n, k) uint32 words
bool stats_needs_sort(const Geometry& g);
size_t sorted_stats_words(int64_t n, int k);
// C64P != nullptr: the SSE residuals are accumulated in the same pass
hipError_t launch_stats_sorted(const float* X, const Geometry& g, const int32_t* labels, double* stats,
                               uint32_t* scratch, const double* C64P, int n_cu, const int* gate, hipStream_t s);
// C64P != nullptr: the SSE residuals are accumulated in the same pass
// C64P, C32 != nullptr: the SSE residuals in the same pass (to the fp32 image,
// corrected per cluster to the float64 centroid at the flush)
hipError_t launch_stats(const float* X, const Geometry& g, const int32_t* labels, double* stats, int n_cu,
                        const int* gate, hipStream_t s, const double* C64P = nullptr, const float* C32 = nullptr);
// stats = [k][d+1] sums and counts, then the SSE slot stats[k (d+1)]
// gate: the batch's stop flag (kernels of later iterations no-op once it is
// set); stop_tol >= 0 lets k_finalize raise it (KM_STOP_*), < 0 never
// dev_repair: empty clusters are repaired on the device (launch_repair), so
// they neither raise the gate nor allow a convergence stop here
// corr: the SSE slot holds residuals to the fp32 images c' (k_s1 delta fit
// with compute_sse); the update adds the exact per-cluster correction
// clear / C32, cmax (one-workgroup update only, update_one_ok): zero the
// statistics after use and write the small path's images of the new centroids
bool update_one_ok(const Geometry& g);
hipError_t launch_update(double* stats, const double* C64_old, const Geometry& g, double* C64_new,
                         double* work, int64_t* counts, const uint32_t* qcount, uint32_t nq, DevStatus* status,
                         int* gate, double stop_tol, int dev_repair, hipStream_t s, int clear = 0,
                         float* C32 = nullptr, float* cmax = nullptr, int corr = 0);
hipError_t launch_sum_x(const float* X, const Geometry& g, double* out, hipStream_t s);
hipError_t launch_scatter_rows(const int64_t* ids, const double* rows, int32_t n, int d, double* C, hipStream_t s);
hipError_t launch_gather_rows(const float* X, const Geometry& g, const int64_t* idx, int32_t n, double* out,
                              hipStream_t s);
// on-device empty-cluster repair after the update of one iteration: the
// Bernoulli passes, then one workgroup for the rest (km_sample.hip); no-ops
// unless the update left empty clusters and the gate is down
hipError_t launch_repair(int* gate, const int64_t* counts, const Geometry& g, int64_t total, double neg_log_delta,
                         uint64_t seed, int32_t* empty, int32_t* pcounts, int64_t* picks, int64_t* samples, int cp,
                         const int64_t* sizes, const int64_t* bases, int nparts, const float* X, int64_t row0,
                         const double* C_old, double* C_new, DevStatus* st, double tol, hipStream_t s);
// the same repair with the rows spread over ranks: pick writes the picked rows
// this context holds into rows[num][d] (zeros for the others) and pending =
// num; the caller sum-all-reduces rows; apply puts them in place
hipError_t launch_repair_pick(int* gate, const int64_t* counts, const Geometry& g, int64_t total,
                              double neg_log_delta, uint64_t seed, int32_t* empty, int32_t* pcounts, int64_t* picks,
                              int64_t* samples, int cp, const int64_t* sizes, const int64_t* bases, int nparts,
                              const float* X, int64_t row0, DevStatus* st, double* rows, int32_t* pending,
                              hipStream_t s);
hipError_t launch_repair_apply(int* gate, const Geometry& g, const int32_t* empty, const double* C_old,
                               double* C_new, DevStatus* st, double tol, const double* rows, const int32_t* pending,
                               hipStream_t s);
// takeSample's Bernoulli pass, one wave per partition (km_sample.hip)
hipError_t launch_bernoulli(const uint64_t* seeds, const int64_t* sizes, const int64_t* bases, int nparts,
                            double fraction, int64_t* out, int cp, int32_t* counts, hipStream_t s);
// One-MFMA screen with in-kernel fp32 re-scoring (km_screen1.hip; the c3
// class): greedy chain colouring (perm: table index -> centroid), the
// per-iteration images, and the screen itself (delta: previous labels read,
// changed rows moved between the float64 sums in `stats`; else labels only)
bool s1_ok(const Geometry& g);
size_t s1_table_entries(const Geometry& g);
hipError_t launch_s1_color(const float* C32, const Geometry& g, int32_t* perm, const int* gate, hipStream_t s);
hipError_t launch_s1_prep(const double* C64, const float* C32, const Geometry& g, const int32_t* perm,
                          const float* cmax, const float* xabs, const float* cabs, float* cft, float* cn2o,
                          uint4* img, float* cst, const int* gate, hipStream_t s);
hipError_t launch_s1(const float* X, const float* xnorm, const Geometry& g, const uint4* img, const float* cn2o,
                     const float* cft, const int32_t* perm, const float* cst, int32_t* labels,
                     QEntry* queue, uint32_t* qcount, uint2* chg, uint32_t* chg_cnt, int delta, int n_cu,
                     QLayout* ql, const int* gate, hipStream_t s, int rev = 0, double* sse = nullptr);
// k_s1's change list: entries (wave segments) and per-wave counts to allocate
size_t s1_chg_entries(const Geometry& g, int n_cu);
size_t s1_wave_slots(int n_cu);
// delta statistics possible (16-bit cluster ids; k_s1_delta aggregates in
// LDS where the [k][d+1] table fits, else with global float64 atomics)
bool s1_delta_ok(const Geometry& g, int n_cu);
// delta statistics: the change list of k_s1 into stats (deltas)
hipError_t launch_s1_delta(const float* X, const Geometry& g, const uint2* chg, const uint32_t* chg_cnt,
                           double* stats, int n_cu, const int* gate, hipStream_t s, const uint32_t* qcount = nullptr);
// the same for any change list of nw wave segments of seg entries
// (k_assign_mfma16's delta mode: its queue layout); qcount != nullptr: each
// segment also holds the resolvers' entries (launch_resolve with delta)
hipError_t launch_chg_delta(const float* X, const Geometry& g, const uint2* chg, const uint32_t* chg_cnt, int nw,
                            uint32_t seg, double* stats, int n_cu, const int* gate, hipStream_t s,
                            const uint32_t* qcount = nullptr);
// delta statistics: mode 1 full += stats, stats = full; mode 0 full = stats
hipError_t launch_s1_apply(double* stats, double* full, int64_t len, int mode, const int* gate, hipStream_t s);
hipError_t launch_gen_blobs(float* X, const Geometry& g, int64_t row_offset, int32_t n_centers, float box,
                            float stddev, uint64_t seed, hipStream_t s);

}  // namespace km
