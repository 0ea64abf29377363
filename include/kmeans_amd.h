/*
 * kmeans_amd.h - C-ABI of the MI355X-native Lloyd-iteration hot path.
 *
 * Drop-in boundary for the reference's per-iteration worker closures and the
 * Spark collectives around them (ersanjay16/Assignment--2-Group7-distributed-K-means,
 * kmeans_spark.py).  The reference has no FFI of its own: its interface for
 * this path is the PySpark RDD calls inside class KMeans, and each entry point
 * below names the reference call it replaces.  The Python host layer
 * (assignment--2-group7-distributed-k-means_amd/kmeans.py) binds these with
 * ctypes and re-exposes the reference's KMeans(...)/fit(rdd, sc)/predict(rdd, sc)
 * surface.
 *
 * Conventions
 *   - every function returns int: 0 = OK (KM_OK), KM_EMPTY (>0) where noted,
 *     < 0 = error; km_last_error() returns a thread-local message.
 *   - plain C types only: host pointers are caller-owned and may be released
 *     when the call returns; device pointers are marked "device".
 *   - all matrices are row-major; centroids are float64 [k][d]; data rows are
 *     float32 [n][d] (stored padded to a multiple of 16 features in HBM).
 *   - one context = one GPU = one rank; a context is not thread-safe.
 *   - work is enqueued on the context stream (km_set_stream, default: own
 *     non-blocking stream); calls that return host data synchronise it.
 */
#ifndef KMEANS_AMD_H
#define KMEANS_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KM_ABI_VERSION 6

#define KM_OK 0
#define KM_EMPTY 1          /* informational: the update found empty clusters */
#define KM_ERR_ARG (-1)
#define KM_ERR_HIP (-2)
#define KM_ERR_STATE (-3)
#define KM_ERR_UNSUPPORTED (-4)

typedef struct km_ctx km_ctx;

/* Per-iteration result of km_update (quantities of kmeans_spark.py:176-313). */
typedef struct km_status {
  double sse;        /* SSE of this assignment w.r.t. the pre-update centroids
                        (replaces _compute_sse, kmeans_spark.py:208-237)        */
  double max_shift;  /* max_c ||new_c - old_c||, empties counted as 0
                        (kmeans_spark.py:293-294)                                */
  int32_t n_empty;   /* clusters absent from the reduce (kmeans_spark.py:186-188) */
  int32_t nonfinite; /* NaN/Inf in a new centroid (kmeans_spark.py:289)         */
  int32_t q_rerank;  /* points whose top-2 were re-ranked in float64             */
  int32_t q_full;    /* points that needed a full float64 scan                   */
  int32_t ran;       /* 1: the iteration ran (0: a no-op of a stopped batch)     */
  int32_t stop_reason; /* KM_STOP_* this iteration raised (batches), else 0     */
  int32_t repaired;  /* its empty clusters were replaced on the device
                        (max_shift includes them, kmeans_spark.py:191-204)      */
  int32_t reserved;
} km_status;

/* Why a batch stopped (km_status.stop_reason). */
#define KM_STOP_CONVERGED 1 /* max_shift < tolerance (kmeans_spark.py:310)       */
#define KM_STOP_EMPTY 2     /* empty clusters: host repair (kmeans_spark.py:191)  */
#define KM_STOP_NONFINITE 3 /* NaN/Inf centroid (kmeans_spark.py:289)            */
/* Iterations per batch (km_batch_begin .. km_batch_end). */
#define KM_MAX_BATCH 32

/* Static facts about a context (for logging / benchmarks). */
typedef struct km_info {
  int64_t n;         /* local rows                                    */
  int32_t d, dp;     /* features, padded row stride                   */
  int32_t k, kp;     /* clusters, padded to a multiple of 64          */
  int32_t path;      /* 1 = small direct-form path, 2 = MFMA fp16x3 screen
                        (k_fused / k_assign_mfma; k_assign_wide for dp > 256) */
  int32_t n_cu;      /* compute units of the device                   */
  int32_t device;
  int32_t fused_stats;
  int32_t delta_stats; /* ABI 6: the last km_assign_stats left changes since the
                          previous assignment in the stats buffer (delta
                          statistics, see km_assign_stats), not full sums */
} km_info;

/* Kernel kinds for km_prof_read. */
#define KM_K_ASSIGN 0
#define KM_K_RESOLVE 1
#define KM_K_STATS 2
#define KM_K_UPDATE 3
#define KM_K_PREP 4
#define KM_K_COUNT 5

int km_abi_version(void);
const char* km_last_error(void);
int km_device_count(int* out);

/* Context lifetime.  Replaces the SparkContext / executor set-up
 * (kmeans_spark.py:626) for one GPU. */
int km_create(int device, km_ctx** out);
int km_destroy(km_ctx* ctx);
/* Enqueue on an external stream (e.g. torch.cuda.current_stream()); NULL =
 * the context's own stream. */
int km_set_stream(km_ctx* ctx, void* hip_stream);
int km_sync(km_ctx* ctx);
int km_info_get(km_ctx* ctx, km_info* out);

/* Materialise this rank's rows in HBM once: replaces sc.parallelize(X) +
 * rdd.cache() (kmeans_spark.py:256, 369, 418, 471, 518, 568).  km_load_begin
 * allocates n rows of d features; km_load_rows copies host float32 rows
 * [row0, row0 + nrows) (pinned staging, chunked). */
int km_load_begin(km_ctx* ctx, int64_t n, int32_t d);
int km_load_rows(km_ctx* ctx, int64_t row0, const float* rows, int64_t nrows);
/* Synthetic Gaussian blobs generated in HBM, keyed by global row (benchmarks). */
int km_generate_blobs(km_ctx* ctx, int64_t n, int32_t d, int64_t global_row0, int32_t n_centers, float box,
                      float stddev, uint64_t seed);
/* Local sum_p x_p of the resident rows (float64 [d]; integrity checks). */
int km_sum_x(km_ctx* ctx, double* out_d);
/* compute_sse (kmeans_spark.py:38, 278-286): when enabled, km_assign_stats
 * also adds every row's float64 residual ||x - c_label||^2 to the SSE slot of
 * the stats buffer, in the same pass over the rows that assigns them
 * (replaces _compute_sse's second pass, :208-237). */
int km_set_sse(km_ctx* ctx, int32_t enable);

/* Set the current centroids: replaces sc.broadcast(self.centroids)
 * (kmeans_spark.py:268, 340). */
int km_set_centroids(km_ctx* ctx, const double* C, int32_t k, int32_t d);
/* Read centroids: which = 0 current, 1 the update's new centroids. */
int km_get_centroids(km_ctx* ctx, int32_t which, double* out);

/* Assignment + partial statistics of one iteration: replaces
 * rdd.mapPartitions(assign_partition) + the map-side combine of
 * reduceByKey (kmeans_spark.py:147-171).  Output = the stats buffer
 * (float64 [k][d+1]: per-cluster sum of x, then count; then one SSE slot,
 * 0 unless km_set_sse is on).
 * Delta statistics (ABI 5, the k_s1 screen's geometries, compute_sse off):
 * from the second iteration after new centroids / rows / a predict, the
 * buffer holds only the CHANGES since the previous assignment (rows that
 * moved: -x, -1 on the old cluster, +x, +1 on the new one), and the context
 * keeps the full sums itself; the update folds the (all-reduced) changes
 * into them.  Summing the buffer over ranks is valid either way (every rank
 * takes the same path: the choice depends on the call sequence and the
 * geometry only).  After a batch update the buffer is zero.  A caller that
 * reads the sums themselves takes the buffer with km_stats_buffer, which
 * turns delta statistics off for the context (full sums every iteration). */
int km_assign_stats(km_ctx* ctx);
/* The stats buffer (device) and its length in doubles, k (d+1) + 1; a caller
 * may bind an external device buffer instead (e.g. a torch tensor it
 * all-reduces): this is the reduceByKey shuffle + collect
 * (kmeans_spark.py:169-173) and the partition-SSE .sum() (:237).
 * km_stats_buffer: the buffer then always holds full sums after
 * km_assign_stats (delta statistics off).  km_bind_stats_buffer keeps delta
 * statistics on: the bound buffer carries the sums or the changes as
 * described at km_assign_stats, which is what a sum all-reduce needs. */
int km_stats_buffer(km_ctx* ctx, void** dev_ptr, int64_t* len);
int km_bind_stats_buffer(km_ctx* ctx, void* dev_ptr);

/* Centroid update from the (all-reduced) stats: replaces _update_centroids
 * (kmeans_spark.py:176-206), reads the SSE slot (:208-237) and computes the
 * shifts (:293-294).  Synchronises; fills *st and counts[k].
 * Returns KM_EMPTY when clusters are empty (their new centroid is the old
 * one until km_replace_rows). */
int km_update(km_ctx* ctx, km_status* st, int64_t* counts);
/* The dataset's partition layout for rdd.takeSample (sizes[nparts] in row
 * order; this context's rows start at global row row0).  device_repair = 1
 * (one context holding every row) moves the empty-cluster repair of
 * kmeans_spark.py:191-204 onto the device inside batches: after an update
 * with empty clusters, takeSample(False, n_empty, empty_seed) runs there
 * (PySpark's fraction, per-partition Bernoulli passes with CPython's MT19937,
 * shuffle; one pass, no retry), its rows replace the empty clusters and their shifts enter
 * max_shift, without stopping the batch (km_status.repaired = 1).  Otherwise
 * (or if a pass overflows its slots or comes back short: the device does not
 * retry PySpark's resampling loop) empty clusters stop the batch and the
 * caller repairs them on the host with the same policy. */
int km_set_layout(km_ctx* ctx, const int64_t* sizes, int32_t nparts, int64_t row0, int32_t device_repair);
/* device_repair = 2 (ABI 4): the rows are spread over ranks, this context
 * holding global rows [row0, row0 + n).  Every rank runs the same takeSample
 * passes over all partitions (index level), so all pick the same rows; then,
 * for an iteration whose km_update_async left the repair waiting
 * (km_repair_state: waiting = 1), the caller sum-all-reduces the repair
 * buffer (km_repair_buffer: k*d doubles, each rank contributing the picked
 * rows it holds and zeros) on the context's stream, and km_repair_apply_async
 * puts the rows in place and finishes the iteration -- no host round trip.
 * Replaces the driver-side takeSample + broadcast of kmeans_spark.py:191-204
 * when the rows sit on several GPUs.  The seed passed to km_update_async must
 * be the same on every rank. */
int km_repair_state(km_ctx* ctx, int32_t* armed, int32_t* waiting);
int km_repair_buffer(km_ctx* ctx, void** buffer, int64_t* len);
/* use an external device buffer of k*d doubles (e.g. a torch tensor that the
 * process group all-reduces); NULL restores the context's own */
int km_bind_repair_buffer(km_ctx* ctx, void* buffer);
int km_repair_apply_async(km_ctx* ctx);
/* Batches of Lloyd iterations without host synchronisation (replaces the
 * per-iteration driver round trip of kmeans_spark.py:266-313).  Between
 * km_batch_begin and km_batch_end the caller enqueues up to KM_MAX_BATCH
 * iterations, each km_assign_stats [+ its all-reduce of the stats buffer] +
 * km_update_async(tol, empty_seed) (empty_seed: int(time.time()), the seed
 * of kmeans_spark.py:196 for an on-device repair); km_update_async also
 * commits speculatively.  The
 * device records every iteration (status, counts) and, on convergence
 * (max_shift < tol), empty clusters or non-finite centroids, raises a gate
 * that turns the rest of the batch into no-ops.  km_batch_end synchronises
 * once, returns the records of the iterations that ran (*n_ran of them:
 * st[i], counts[i*k .. i*k+k)) and leaves the context as km_update would
 * after the last of them: km_replace_rows / km_commit apply to it. */
int km_batch_begin(km_ctx* ctx);
int km_update_async(km_ctx* ctx, double tol, int64_t empty_seed);
int km_batch_end(km_ctx* ctx, km_status* st, int64_t* counts, int32_t* n_ran);
/* Empty-cluster repair (kmeans_spark.py:196-204): overwrite new centroids
 * of the given clusters with the given rows (float64 [n][d]). */
int km_replace_rows(km_ctx* ctx, const int32_t* cluster_ids, const double* rows, int32_t n);
/* Commit the new centroids (kmeans_spark.py:307). */
int km_commit(km_ctx* ctx);

/* Rows by local index (float64 [n][d]): the rows behind rdd.takeSample
 * (kmeans_spark.py:72, 196). */
int km_gather_rows(km_ctx* ctx, const int64_t* local_idx, int32_t n, double* out);

/* Bernoulli pass of rdd.takeSample(False, num, seed) (kmeans_spark.py:72,
 * 196; PySpark RDD.takeSample + RDDSampler): for each of the nparts given
 * partitions, row i is kept when the i-th double of Python's
 * random.Random(seeds[p]) (seeds[p] = takeSample seed ^ partition index,
 * after ten randint(0, 1) warm-up draws) is < fraction.  One wave per
 * partition on this context's GPU.  out[0..*n_out): global row indices
 * bases[p] + i, partitions in the given order, rows ascending.  KM_ERR_ARG
 * when a partition yields more picks than the device pass holds (4x the
 * expectation + 64) or *n_out would exceed cap: the caller then samples on
 * the host. */
int km_bernoulli_sample(km_ctx* ctx, const uint64_t* seeds, const int64_t* sizes, const int64_t* bases,
                        int32_t nparts, double fraction, int64_t* out, int64_t cap, int64_t* n_out);

/* Labels of every local row for the current centroids: replaces predict's
 * assign_partition (kmeans_spark.py:343-350). */
int km_predict(km_ctx* ctx, int32_t* labels_out);
/* Labels of the last km_assign_stats (device -> host). */
int km_labels(km_ctx* ctx, int32_t* labels_out);

/* Screening kernel.  A cost choice: labels, sums and SSE are exact in every
 * mode.  -1 (default): the one-MFMA screen k_s1 (mode 4) wherever the
 * geometry has an instance, else mode 5 on the unfused path (dp a multiple
 * of 32), else per batch from the last iteration's queue fraction; 0: fp16x3
 * screen, global bound; 1: fp16x3 with per-key bounds (0 and 1 keep
 * k_fused16 with full statistics on every iteration, and the fp16x3
 * k_assign_mfma16 on the unfused path); 4 (ABI 5): k_s1, one fp16 MFMA per
 * product, candidates re-scored exactly in fp32 inside the kernel, delta
 * statistics on the fused geometries (the first iteration after new data,
 * centroids or a predict still runs the fp16x3 screen with full statistics;
 * with compute_sse every iteration does), labels then the statistics pass on
 * the unfused ones; 5 (ABI 5): one fp16 MFMA per product in the unfused
 * k_assign_mfma16 with the one-part bound, the rows it cannot settle going
 * to the float64 resolvers (candidate lists).  Modes 2 and 3 (fast screen:
 * one fp16 MFMA per product, pairwise bound; 3 with the row split hi + lo)
 * exist in the diagnostic library only (libkmeans_amd_diag.so, make diag);
 * the product library returns KM_ERR_UNSUPPORTED for them. */
#define KM_SCREEN_AUTO (-1)
#define KM_SCREEN_S1 4
#define KM_SCREEN_ONE 5
int km_set_screen(km_ctx* ctx, int32_t mode);
/* The screen the next assign with statistics uses (0..5). */
int km_get_screen(km_ctx* ctx, int32_t* mode);

/* Kernel timing with HIP events on the context stream.  `enable` is a
 * bitmask of (1 << KM_K_*) phases to time (-1: all, 0: off). */
int km_profile(km_ctx* ctx, int32_t enable);
/* Time one launch in `period` (>= 1, default 1) of each profiled phase: each
 * timed launch costs ~6 us of stream time, which a 0.16 ms c2 step notices. */
int km_profile_every(km_ctx* ctx, int32_t period);
int km_prof_read(km_ctx* ctx, int32_t kind, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* KMEANS_AMD_H */
