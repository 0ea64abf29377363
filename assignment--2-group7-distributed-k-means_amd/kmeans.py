"""``KMeans`` — drop-in for the reference's class (kmeans_spark.py:19-352).

Same constructor, attributes, messages, log lines and iteration order as the
reference; the Lloyd iteration itself runs on the GPU (``engine.HipEngine``):

  reference (PySpark)                         here
  -------------------------------------       -----------------------------------------
  rdd.cache()                      L256       rows copied to HBM once (engine.load_*)
  sc.broadcast(centroids)          L268       centroids already resident (commit)
  mapPartitions(assign_partition)  L161-171   km_assign_stats (screen + exact resolve + stats)
  reduceByKey(..).collect()        L169-173   one RCCL all-reduce of the [k][d+1] stats
  _update_centroids                L176-206   km_update (+ host empty-cluster repair)
  _compute_sse                     L208-237   float64 residual of every row, same pass (SSE slot)
  NaN check / shift / log / commit L289-313   identical, from the device status

There is no CPU fallback: without the HIP extension or a gfx950 GPU, ``fit``
and ``predict`` raise ``RuntimeError``.
"""
from __future__ import annotations

import sys
import time
import weakref
from typing import List, Optional

import numpy as np

from . import _lib, sampling
from .comm import Communicator
from .dataset import DeviceBlobs, EmptyDataset, LocalRDD, Placement, place
from .engine import make_engine


class LloydRunner:
    """Engine + data placement + communicator of one ``fit``; ``iteration``
    performs one Lloyd iteration exactly as kmeans_spark.py:266-318."""

    def __init__(self, engine, placement: Placement, comm: Communicator, k: int):
        self.engine = engine
        self.pl = placement
        self.comm = comm
        self.k = k
        self.last = None
        self.device_repairs = 0  # iterations whose empty clusters the device replaced
        self.iterations_ran = 0  # iterations the device ran in batches (bench.py divides by these)
        self.host_ms = None      # {call kind: host wall ms} while a caller times run() (bench.py)
        # takeSample's Bernoulli pass on the GPU when the engine has one
        self.sampler = getattr(engine, "bernoulli", None)

    # -- set-up --------------------------------------------------------------------
    def load(self) -> None:
        pl = self.pl
        if pl.blobs is not None:
            b = pl.blobs
            self.engine.load_blobs(pl.n_local, b.d, pl.row0, b.n_centers, b.box, b.std, b.seed)
        else:
            self.engine.load_host(pl.local_rows)
        # empty clusters are repaired on the device (takeSample policy,
        # kmeans_spark.py:191-204) without stopping a batch: mode 1 with one
        # rank holding every row; mode 2 with the rows spread over ranks (every
        # rank picks the same rows, the owners contribute them to one
        # stream-ordered all-reduce, LloydRunner.run)
        self.device_repair = 0
        if hasattr(self.engine, "set_layout"):
            if self.comm.world == 1:
                self.device_repair = 1
            elif hasattr(self.engine, "repair_exchange") and getattr(self.engine, "distributed", False):
                self.device_repair = 2
        if self.device_repair:
            self.engine.set_layout(pl.global_sizes, pl.row0 if self.device_repair == 2 else 0, self.device_repair)

    def rows(self, gidx: List[int]) -> np.ndarray:
        """Rows by global index (what ``rdd.takeSample`` returns, L72/L196):
        each rank gathers the ones it holds from HBM (the stored float32 rows,
        as float64), one sum all-reduce assembles them (others contribute 0)."""
        gidx = np.asarray(gidx, dtype=np.int64)
        lo, hi = self.pl.row0, self.pl.row0 + self.pl.n_local
        mine = np.nonzero((gidx >= lo) & (gidx < hi))[0]
        out = np.zeros((len(gidx), self.pl.d), dtype=np.float64)
        if len(mine):
            out[mine] = self.engine.gather_rows(gidx[mine] - lo)
        return self.comm.allreduce_np(out)

    # -- Lloyd iterations ---------------------------------------------------------------
    batch = 4  # first batch size; doubles (to KM_MAX_BATCH) while batches run through

    def run(self, model: "KMeans", log, max_iter: int, first: int = 0) -> bool:
        """Iterations ``first .. max_iter-1`` of the loop of kmeans_spark.py:266-313,
        in batches: per iteration assign + stats, the all-reduce and the update are
        enqueued without host synchronisation; the device records each
        iteration and stops the batch on convergence, empty clusters or
        non-finite centroids.  The host then replays, from those records, the
        per-iteration log lines and SSE history, and handles the last iteration
        that ran exactly as ``iteration`` does.  Returns True on convergence."""
        it = first
        eng = self.engine
        # host wall time per call kind (bench.py's N > 1 lines): None = off
        ht = self.host_ms
        clk = time.perf_counter
        # the batch size carries over between calls on one runner (a caller
        # running the loop in pieces, like bench.py's warmup and timed region)
        size = getattr(self, "_next_batch", self.batch)
        while it < max_iter:
            m = min(size, max_iter - it)
            # the repair seed of each iteration, int(time.time()) read per
            # iteration as L196 reads it per repair
            seeds = [model._empty_seed() for _ in range(m)]
            t = clk()
            if self.device_repair == 2:
                eng.repair_bind()
                if eng.repair_state()[0]:                      # armed: every rank needs the same seeds
                    seeds = self.comm.broadcast_obj(seeds)
            eng.batch_begin()
            if ht is not None:
                ht["batch_begin"] = ht.get("batch_begin", 0.0) + (clk() - t) * 1e3
            try:
                for b in range(m):
                    t0 = clk()
                    eng.assign_stats()                         # L272 (+ L169-171 map side)
                    t1 = clk()
                    self.comm.allreduce_stats(eng)             # L169-173 shuffle + collect
                    t2 = clk()
                    # L176-206 (+ the repair's seed, L196), device convergence test
                    eng.update_async(model.tolerance, seeds[b])
                    t3 = clk()
                    if self.device_repair == 2 and eng.repair_state()[1]:
                        # the picked rows from their owners (L196-200), then the rest
                        # of the update on the device
                        eng.repair_exchange(self.comm.dist.all_reduce)
                    if ht is not None:
                        t4 = clk()
                        for key, v in (("assign_stats", t1 - t0), ("allreduce", t2 - t1),
                                       ("update_async", t3 - t2), ("repair", t4 - t3)):
                            ht[key] = ht.get(key, 0.0) + v * 1e3
            except BaseException:
                # close the batch (the gate comes down, the context is back to
                # the last iteration that ran), then report the original error
                try:
                    eng.batch_end(m)
                except Exception:
                    pass
                raise
            t = clk()
            recs = eng.batch_end(m)
            if ht is not None:
                ht["batch_end"] = ht.get("batch_end", 0.0) + (clk() - t) * 1e3
            self.iterations_ran += len(recs)
            # a batch that ran through doubles the next one (fewer host round
            # trips on long runs); a stopped one (convergence, empties) resets it
            size = min(2 * size, _lib.KM_MAX_BATCH) if len(recs) == m and not recs[-1][0].stop_reason else self.batch
            self._next_batch = size
            for b, (st, counts) in enumerate(recs):
                if b + 1 < len(recs):                          # ran through: committed on the device
                    self._record(model, it, st, counts, st.max_shift, log)
                elif self._after_update(model, it, st, counts, log):
                    return True
                it += 1
        return False

    def iteration(self, model: "KMeans", iteration: int, log) -> bool:
        """One Lloyd iteration with a host sync (kmeans_spark.py:266-318).
        Returns True when converged (max_shift < tolerance)."""
        eng = self.engine
        eng.assign_stats()                                     # L272 (+ L169-171 map side)
        self.comm.allreduce_stats(eng)                         # L169-173 shuffle + collect
        st, counts = eng.update()                              # L176-188 (+ SSE, shift)
        return self._after_update(model, iteration, st, counts, log)

    def _record(self, model, iteration, st, counts, max_shift, log) -> None:
        """An iteration that ran through on the device: the empty-cluster
        warning if the device repaired some (L192), SSE history with its
        warning (L278-286), then the log line (L297-304)."""
        if st.n_empty:
            self.device_repairs += 1
            if log:
                log(f"  WARNING: {int(st.n_empty)} empty cluster(s) detected. Reinitializing...")
        self._sse(model, st, log)
        self._log_line(model, iteration, st, counts, max_shift, log)

    @staticmethod
    def _sse(model, st, log) -> None:
        if model.compute_sse:                                  # L278-286
            sse = float(st.sse)
            model.sse_history.append(sse)
            if log and len(model.sse_history) > 1 and sse > model.sse_history[-2] + 1e-6:
                log(f"  WARNING: SSE increased from {model.sse_history[-2]:.4f} to {sse:.4f}")

    def _log_line(self, model, iteration, st, counts, max_shift, log) -> None:
        if log:  # None when nothing is printed (not verbose, or not rank 0): skip the formatting
            cluster_sizes = [int(c) for c in counts]           # L297
            if model.compute_sse and model.sse_history:
                log(f"Iteration {iteration + 1}: SSE = {model.sse_history[-1]:.4f}, "
                    f"Max Shift = {max_shift:.6f}, Cluster Sizes = {cluster_sizes}")
            else:
                log(f"Iteration {iteration + 1}: Max Shift = {max_shift:.6f}, Cluster Sizes = {cluster_sizes}")
        self.last = {"max_shift": max_shift, "sse": float(st.sse) if model.compute_sse else None,
                     "counts": counts, "n_empty": int(st.n_empty), "q_rerank": int(st.q_rerank),
                     "q_full": int(st.q_full)}

    def _after_update(self, model, iteration, st, counts, log) -> bool:
        """The rest of an iteration once the device update is done (state: new
        centroids computed, not committed): empty repair, SSE, NaN check, log,
        commit, convergence (kmeans_spark.py:191-313)."""
        eng, k = self.engine, self.k
        max_shift = st.max_shift
        nonfinite = bool(st.nonfinite)
        if st.n_empty and getattr(st, "repaired", 0):          # L191-204 done on the device
            self.device_repairs += 1
            if log:
                log(f"  WARNING: {int(st.n_empty)} empty cluster(s) detected. Reinitializing...")
        elif st.n_empty:                                       # L191
            empty = [j for j in range(k) if counts[j] == 0]
            if log:
                log(f"  WARNING: {len(empty)} empty cluster(s) detected. Reinitializing...")
            seed = self.comm.broadcast_obj(model._empty_seed())    # int(time.time()), L196
            gidx = sampling.take_sample(self.pl.global_sizes, len(empty), seed, self.comm, self.sampler)
            reps = self.rows(gidx) if gidx else np.zeros((0, self.pl.d))
            old = eng.get_centroids(0)
            ids = empty[:len(reps)]                            # the rest keep the old centroid (L204)
            if ids:
                eng.replace_rows(ids, reps)
                shift = np.linalg.norm(reps[:len(ids)] - old[ids], axis=1)
                max_shift = max(max_shift, float(np.max(shift)))
                nonfinite = nonfinite or not np.all(np.isfinite(reps))
        self._sse(model, st, log)                              # L278-286
        if nonfinite:                                          # L289-290
            raise ValueError(f"NaN or Inf detected in centroids at iteration {iteration + 1}")
        self._log_line(model, iteration, st, counts, max_shift, log)   # L293-304
        eng.commit()                                           # L307
        if max_shift < model.tolerance:                        # L310-313
            if log:
                log(f"Converged after {iteration + 1} iterations")
            return True
        return False


class LabelsRDD(LocalRDD):
    """``predict``'s result: an RDD-like of Python ints in input order.

    The labels stay sharded (each rank holds its own rows' labels, its row
    block of the input) until an action needs them:

    * ``collect()`` / ``to_numpy()`` bring them to the driver, as Spark's
      collect() does: rank 0 gathers every rank's shard (one gather of N
      int32, not an all-gather of N per rank), the other ranks get ``[]`` /
      an empty array.  ``everywhere=True`` (per call, or for the object at
      construction) gives every rank the whole list (one all-gather);
    * ``count()`` sums the shard lengths;
    * ``local()`` is this rank's shard with no communication;
    * the other RDD methods inherited from ``LocalRDD`` (``glom``,
      ``mapPartitions``, ``partition_array`` ...) run without communication
      on this rank's shard (one partition), or on every label once
      ``collect(everywhere=True)`` gathered them; with one rank that is the
      whole result."""

    def __init__(self, local_labels: np.ndarray, comm: Communicator, everywhere: bool = False):
        self._local = local_labels
        self._comm = comm
        self._everywhere = everywhere
        self._all = None     # every rank's labels (everywhere)
        self._root = None    # the driver's copy (rank 0)
        super().__init__([])

    @property
    def _parts(self):
        # what the inherited LocalRDD methods see (never a collective: an
        # inherited method may run on one rank only)
        return [self._all if self._all is not None else self._local]

    @_parts.setter
    def _parts(self, value):  # LocalRDD.__init__ assigns it; the labels are the data
        pass

    def _gather(self, everywhere: Optional[bool]) -> np.ndarray:
        ev = self._everywhere if everywhere is None else everywhere
        if self._comm.world == 1:
            return self._local
        if ev:
            if self._all is None:
                self._all = np.concatenate(self._comm.allgather_array(self._local))
            return self._all
        if self._all is not None:
            return self._all if self._comm.rank == 0 else self._local[:0]
        if self._root is None:
            parts = self._comm.gather_array(self._local, root=0)
            self._root = np.concatenate(parts) if parts is not None else self._local[:0]
        return self._root

    def collect(self, everywhere: Optional[bool] = None) -> list:
        return self._gather(everywhere).tolist()

    def count(self) -> int:
        if self._comm.world > 1:
            return int(self._comm.allreduce_np(np.array([float(len(self._local))]))[0])
        return int(len(self._local))

    def getNumPartitions(self) -> int:
        return self._comm.world

    def local(self) -> np.ndarray:
        """This rank's labels (rows [row0, row0 + n_local) of the input)."""
        return self._local

    def to_numpy(self, everywhere: Optional[bool] = None) -> np.ndarray:
        return self._gather(everywhere)


def _ref_to(obj):
    """A reference to the fitted dataset for predict's reuse test: weak where
    the type allows (the model does not keep the host data alive), else the
    object itself.  Compared by identity (``is``), never by ``id()``, which
    CPython reuses after garbage collection."""
    try:
        return weakref.ref(obj)
    except TypeError:
        return lambda: obj


def _deref(ref):
    return ref() if ref is not None else None


class KMeans:
    """Distributed K-Means, MI355X-native (kmeans_spark.py:19-47).

    Parameters: k, max_iter, tolerance (max centroid shift), seed (sampling of
    the initial centroids), compute_sse (track the SSE each iteration).

    Compute contract: rows are stored in HBM as float32, rounded once at load
    (a float64 input is not copied at full precision); every row the fit uses
    afterwards -- assignment, per-cluster sums, the takeSample initial and
    replacement centroids -- is that rounded row, and all arithmetic on it
    (distances to decide labels, sums, centroids, SSE) is float64 with the
    reference's NumPy rounding where it decides a label.  The result is
    therefore the reference's result on ``X.astype(float32)``: identical for
    float32-representable data, within float32 rounding (~1e-7 relative of the
    data scale) of the reference on raw float64 rows.  Centroids are returned
    in the input's float dtype."""

    _engine_factory = None  # test seam: tests/ inject a CPU engine for host-logic tests

    def __init__(self, k: int = 3, max_iter: int = 100, tolerance: float = 1e-4,
                 seed: int = 42, compute_sse: bool = False):
        self.k = k
        self.max_iter = max_iter
        self.tolerance = tolerance
        self.seed = seed
        self.compute_sse = compute_sse
        self.centroids: np.ndarray = None
        self.sse_history: List[float] = []
        self._validate_parameters()
        self.iterations_run = 0  # kept as the reference leaves it (never updated, L47)
        self._runner: Optional[LloydRunner] = None
        self._runner_src = None  # the fitted dataset (weak reference where the type allows)
        self.verbose = True

    def _validate_parameters(self):
        if self.k <= 0:
            raise ValueError(f"k must be positive, got {self.k}")
        if self.max_iter <= 0:
            raise ValueError(f"max_iter must be positive, got {self.max_iter}")
        if self.tolerance <= 0:
            raise ValueError(f"tolerance must be positive, got {self.tolerance}")

    # -- hooks -----------------------------------------------------------------------
    def _empty_seed(self) -> int:
        return int(time.time())  # kmeans_spark.py:196

    def _log(self, comm: Communicator):
        """The line printer of this run, or None when nothing would be printed."""
        if not (self.verbose and comm.rank == 0):
            return None

        def say(msg: str):
            print(msg)
            sys.stdout.flush()
        return say

    def _make_runner(self, rdd, comm: Communicator) -> LloydRunner:
        pl = place(rdd, comm)
        factory = type(self)._engine_factory or make_engine
        eng = factory(comm)
        run = LloydRunner(eng, pl, comm, self.k)
        run.load()
        return run

    def _initialize_centroids(self, run: LloydRunner) -> np.ndarray:
        """kmeans_spark.py:58-82: k distinct rows by the takeSample policy."""
        gidx = sampling.take_sample(run.pl.global_sizes, self.k, self.seed, run.comm, run.sampler)
        if len(gidx) < self.k:
            raise ValueError(f"Not enough data points ({len(gidx)}) to initialize {self.k} clusters")
        centroids = np.array(run.rows(gidx))
        if not np.all(np.isfinite(centroids)):
            raise ValueError("Data contains NaN or Inf values")
        return centroids

    # -- public API ----------------------------------------------------------------------
    def fit(self, rdd, sc=None) -> "KMeans":
        if hasattr(rdd, "cache"):
            rdd.cache()                                        # L256
        comm = Communicator()
        try:
            run = self._make_runner(rdd, comm)
        except EmptyDataset:
            # takeSample of an empty RDD returns [] (L72-74)
            raise ValueError(f"Not enough data points (0) to initialize {self.k} clusters") from None
        self._runner, self._runner_src = run, _ref_to(rdd)
        self.centroids = self._initialize_centroids(run)       # L259
        self.sse_history = []                                  # L260
        say = self._log(comm)
        if say:
            say(f"Starting K-Means with k={self.k}, max_iter={self.max_iter}, tolerance={self.tolerance}")
            say(f"SSE computation: {'ENABLED' if self.compute_sse else 'DISABLED (for performance)'}")
        out_dtype = run.pl.dtype
        run.engine.set_centroids(np.asarray(self.centroids, dtype=np.float64))
        run.engine.set_sse(self.compute_sse)
        try:
            run.run(self, say, self.max_iter)                  # L266-313
        finally:
            self.centroids = run.engine.get_centroids(0).astype(out_dtype, copy=False)
        return self

    def predict(self, rdd, sc=None):
        if self.centroids is None:
            raise ValueError("Model must be fitted before prediction")
        comm = Communicator()
        if self._runner is not None and _deref(self._runner_src) is rdd:
            run = self._runner  # the rows are resident from fit
        else:
            try:
                run = self._make_runner(rdd, comm)
            except EmptyDataset:
                return LabelsRDD(np.zeros(0, dtype=np.int32), comm)  # a lazy map over no rows (L350)
        run.engine.set_centroids(np.asarray(self.centroids, dtype=np.float64))
        labels = LabelsRDD(run.engine.predict(), comm)
        if sc is not None and hasattr(sc, "_jsc") and hasattr(rdd, "getNumPartitions"):
            # a real SparkContext (every rank's driver program parallelizes the whole list)
            return sc.parallelize(labels.collect(everywhere=True), rdd.getNumPartitions())
        return labels
