"""CPU restatement (oracle) of the reference Lloyd iteration.

TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product
path (``assignment--2-group7-distributed-k-means_amd``) never imports it.

Every function restates ``/root/reference/kmeans_spark.py`` (cited file:line)
in NumPy, float64, with the reference's own reduction orders so that results
are bit-identical to the reference run under the in-memory PySpark stand-in
(``tests/golden/_pyspark_stub``):

* distance      ``np.linalg.norm(C - x, axis=1)``            kmeans_spark.py:153,231,347
* assignment    ``np.argmin`` (first minimum wins)            kmeans_spark.py:156,348
* partial stats ``reduceByKey(lambda a,b: (a0+b0, a1+b1))``   kmeans_spark.py:169-173
                (left fold inside a partition, partitions merged in order)
* update        ``sum / count``; empties -> takeSample rows   kmeans_spark.py:176-206
* SSE           ``sum(min(norm)**2)`` per partition, summed   kmeans_spark.py:224-237
* loop tail     SSE warning, NaN check, max shift, converge   kmeans_spark.py:266-319
* init          ``rdd.takeSample(False, k, seed)``            kmeans_spark.py:72-80

Pinning: ``tests/test_oracle_golden.py`` checks this module against the golden
vectors in ``tests/golden/*.npz`` that ``tests/golden/make_golden.py``
produced by importing the reference module itself.
"""
from __future__ import annotations

import math
import random
import sys
from typing import Callable, Dict, List, Optional, Sequence

import numpy as np

__all__ = [
    "partition_bounds", "take_sample_indices", "distances", "assign",
    "assign_faithful", "partition_stats", "merge_stats", "update_centroids",
    "partition_sse", "lloyd_fit", "predict",
]


# ---------------------------------------------------------------------------
# data layout helpers
# ---------------------------------------------------------------------------
def partition_bounds(n: int, num_slices: int) -> List[tuple]:
    """Contiguous slices of ``sc.parallelize(X, numSlices)`` (PySpark)."""
    return [((i * n) // num_slices, ((i + 1) * n) // num_slices) for i in range(num_slices)]


def _fraction_for_sample_size(num: int, total: int) -> float:
    fraction = float(num) / total
    delta = 0.00005
    gamma = -math.log(delta) / total
    return min(1.0, fraction + gamma + math.sqrt(gamma * gamma + 2 * gamma * fraction))


def take_sample_indices(partition_sizes: Sequence[int], num: int, seed: Optional[int]) -> List[int]:
    """Index-level restatement of ``rdd.takeSample(False, num, seed)``.

    Reference call sites: kmeans_spark.py:72 (init, ``seed=self.seed``) and
    kmeans_spark.py:196 (empty clusters, ``seed=int(time.time())``).  Follows
    PySpark's algorithm (count, fraction, per-partition Bernoulli sampler
    seeded ``seed ^ split`` with 10 warm-up draws, retry, shuffle, truncate).
    Returns global row indices in the order takeSample would return rows.
    """
    if num < 0:
        raise ValueError("Sample size cannot be negative.")
    if num == 0:
        return []
    total = int(sum(partition_sizes))
    if total == 0:
        return []
    if seed is None:
        seed = random.randint(0, sys.maxsize)
    rand = random.Random(seed)
    if num >= total:
        idx = list(range(total))
        rand.shuffle(idx)
        return idx
    fraction = _fraction_for_sample_size(num, total)

    def one_pass(s):
        out = []
        base = 0
        for split, size in enumerate(partition_sizes):
            rng = random.Random(s ^ split)
            for _ in range(10):
                rng.randint(0, 1)
            for i in range(size):
                if rng.random() < fraction:
                    out.append(base + i)
            base += size
        return out

    samples = one_pass(seed)
    while len(samples) < num:
        seed = rand.randint(0, sys.maxsize)
        samples = one_pass(seed)
    rand.shuffle(samples)
    return samples[0:num]


# ---------------------------------------------------------------------------
# map phase
# ---------------------------------------------------------------------------
def assign_faithful(points: np.ndarray, C: np.ndarray):
    """Per-point loop exactly as ``assign_partition`` (kmeans_spark.py:147-159).
    Returns (labels int64, min distances float64)."""
    labels = np.empty(len(points), dtype=np.int64)
    mind = np.empty(len(points), dtype=np.float64)
    for i, point in enumerate(points):
        dist = np.linalg.norm(C - point, axis=1)          # L153
        labels[i] = int(np.argmin(dist))                 # L156
        mind[i] = np.min(dist)                           # L232
    return labels, mind


def distances(X: np.ndarray, C: np.ndarray, chunk: int = 4096) -> np.ndarray:
    """Vectorised ``np.linalg.norm(C - x, axis=1)`` for every row of X.

    Reduces the contiguous last axis with NumPy's pairwise add.reduce, the
    same kernel ``linalg.norm`` uses for one point (kmeans_spark.py:153), so
    values are bit-identical to the per-point form (checked in tests)."""
    n = X.shape[0]
    out = np.empty((n, C.shape[0]), dtype=np.result_type(X, C))
    for s in range(0, n, chunk):
        diff = C[None, :, :] - X[s:s + chunk, None, :]
        out[s:s + chunk] = np.sqrt(np.add.reduce(diff * diff, axis=-1))
    return out


def assign(X: np.ndarray, C: np.ndarray, chunk: int = 4096):
    """(labels, min-distance, top-2 relative gap) for every row of X."""
    n = X.shape[0]
    labels = np.empty(n, dtype=np.int64)
    mind = np.empty(n, dtype=np.float64)
    gap = np.full(n, np.inf)
    k = C.shape[0]
    for s in range(0, n, chunk):
        D = distances(X[s:s + chunk], C, chunk)
        lab = np.argmin(D, axis=1)
        labels[s:s + chunk] = lab
        mind[s:s + chunk] = D[np.arange(len(lab)), lab]
        if k > 1:
            part = np.partition(D, 1, axis=1)
            d1, d2 = part[:, 0], part[:, 1]
            with np.errstate(divide="ignore", invalid="ignore"):
                gap[s:s + chunk] = np.where(d2 > 0, (d2 - d1) / d2, 0.0)
    return labels, mind, gap


# ---------------------------------------------------------------------------
# reduce phase
# ---------------------------------------------------------------------------
def partition_stats(Xp: np.ndarray, labels: np.ndarray, k: int) -> Dict[int, tuple]:
    """Map-side combine of one partition: left fold of ``(x, 1)`` per key in
    point order (``reduceByKey`` lambda, kmeans_spark.py:169-171)."""
    out = {}
    for c in np.unique(labels):
        pts = Xp[labels == c]
        out[int(c)] = (np.cumsum(pts, axis=0)[-1], int(len(pts)))
    return out


def merge_stats(per_partition: List[Dict[int, tuple]]) -> Dict[int, tuple]:
    """Merge combiners in partition order (reduceByKey + collect, L169-174)."""
    out: Dict[int, tuple] = {}
    for d in per_partition:
        for key in sorted(d):
            s, n = d[key]
            if key in out:
                out[key] = (out[key][0] + s, out[key][1] + n)
            else:
                out[key] = (s, n)
    return out


def update_centroids(cluster_dict, old: np.ndarray, replacement_rows: Callable[[int], np.ndarray],
                     log: Optional[Callable[[str], None]] = None):
    """``_update_centroids`` tail (kmeans_spark.py:176-206).
    ``replacement_rows(n)`` plays ``rdd.takeSample(False, n, seed=int(time.time()))``."""
    k = old.shape[0]
    new = np.zeros_like(old)                                   # L176
    counts = {}
    empty = []
    for cid in range(k):                                       # L181
        if cid in cluster_dict:
            s, n = cluster_dict[cid]
            new[cid] = s / n                                   # L184
            counts[cid] = n
        else:
            empty.append(cid)
            counts[cid] = 0
    if empty:                                                  # L191
        if log:
            log(f"  WARNING: {len(empty)} empty cluster(s) detected. Reinitializing...")
        rows = replacement_rows(len(empty))                    # L196
        for i, cid in enumerate(empty):
            if i < len(rows):
                new[cid] = rows[i]                             # L200
            else:
                new[cid] = old[cid]                            # L204
    return new, counts, empty


def partition_sse(mind: np.ndarray) -> float:
    """``compute_partition_sse`` (kmeans_spark.py:224-235): sequential
    ``partition_sse += min_distance ** 2`` starting from 0.0."""
    if len(mind) == 0:
        return 0.0
    # ``np.float64 ** 2`` on a scalar goes through libm pow(), which is not
    # always the correctly rounded x*x that the array power gives; math.pow
    # is the same libm call, so the squares are bit-identical to L233.
    sq = np.fromiter((math.pow(v, 2) for v in mind.tolist()), dtype=np.float64, count=len(mind))
    return float(np.cumsum(sq)[-1])


# ---------------------------------------------------------------------------
# driver loop
# ---------------------------------------------------------------------------
def lloyd_fit(X: np.ndarray, k: int, max_iter: int = 100, tolerance: float = 1e-4, seed: int = 42,
              compute_sse: bool = False, num_slices: int = 1, init_centroids: Optional[np.ndarray] = None,
              empty_seed: Callable[[], int] = lambda: 0, log: Optional[Callable[[str], None]] = None,
              faithful: bool = False) -> dict:
    """Restates ``KMeans.fit`` (kmeans_spark.py:239-319).

    ``num_slices``: partition count of ``sc.parallelize(X, num_slices)``.
    ``init_centroids``: inject initial centroids (else takeSample restatement, L72).
    ``empty_seed``: replaces ``int(time.time())`` at L196.
    Returns a dict with centroids, sse_history, per-iteration records.
    """
    if k <= 0:
        raise ValueError(f"k must be positive, got {k}")
    if max_iter <= 0:
        raise ValueError(f"max_iter must be positive, got {max_iter}")
    if tolerance <= 0:
        raise ValueError(f"tolerance must be positive, got {tolerance}")
    n = X.shape[0]
    bounds = partition_bounds(n, num_slices)
    sizes = [b - a for a, b in bounds]
    if init_centroids is None:
        idx = take_sample_indices(sizes, k, seed)              # L72
        if len(idx) < k:
            raise ValueError(f"Not enough data points ({len(idx)}) to initialize {k} clusters")
        centroids = np.array(X[idx])
        if not np.all(np.isfinite(centroids)):
            raise ValueError("Data contains NaN or Inf values")
    else:
        centroids = np.array(init_centroids, dtype=X.dtype, copy=True)
    init = centroids.copy()
    sse_history: List[float] = []
    records = []
    say = log or (lambda s: None)
    say(f"Starting K-Means with k={k}, max_iter={max_iter}, tolerance={tolerance}")
    say(f"SSE computation: {'ENABLED' if compute_sse else 'DISABLED (for performance)'}")
    converged = False
    for iteration in range(max_iter):                          # L266
        per_part = []
        part_sse = []
        for a, b in bounds:
            Xp = X[a:b]
            if faithful:
                lab, mind = assign_faithful(Xp, centroids)
            else:
                lab, mind, _ = assign(Xp, centroids)
            per_part.append(partition_stats(Xp, lab, k))
            part_sse.append(partition_sse(mind))
        cluster_dict = merge_stats(per_part)

        def rows(nr):
            gidx = take_sample_indices(sizes, nr, empty_seed())
            return [X[i] for i in gidx]

        new, counts, empty = update_centroids(cluster_dict, centroids, rows, say)
        sse = None
        if compute_sse:                                        # L278
            total = 0
            for s in part_sse:
                total = total + s
            sse = total
            sse_history.append(sse)
            if len(sse_history) > 1 and sse > sse_history[-2] + 1e-6:
                say(f"  WARNING: SSE increased from {sse_history[-2]:.4f} to {sse:.4f}")
        if not np.all(np.isfinite(new)):                       # L289
            raise ValueError(f"NaN or Inf detected in centroids at iteration {iteration + 1}")
        shifts = np.linalg.norm(new - centroids, axis=1)       # L293
        max_shift = np.max(shifts)
        sizes_list = [counts.get(i, 0) for i in range(k)]
        if compute_sse and sse_history:
            say(f"Iteration {iteration + 1}: SSE = {sse_history[-1]:.4f}, "
                f"Max Shift = {max_shift:.6f}, Cluster Sizes = {sizes_list}")
        else:
            say(f"Iteration {iteration + 1}: Max Shift = {max_shift:.6f}, Cluster Sizes = {sizes_list}")
        records.append({"max_shift": float(max_shift), "sizes": sizes_list, "empty": list(empty), "sse": sse})
        centroids = new                                        # L307
        if max_shift < tolerance:                              # L310
            say(f"Converged after {iteration + 1} iterations")
            converged = True
            break
    return {"centroids": centroids, "init": init, "sse_history": sse_history, "records": records,
            "n_iter": len(records), "converged": converged}


def predict(X: np.ndarray, C: np.ndarray) -> np.ndarray:
    """``predict`` (kmeans_spark.py:343-350): ``int(np.argmin(norm))`` per point."""
    return assign(X, C)[0]
