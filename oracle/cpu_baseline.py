"""CPU baseline leg of bench.py (TEST/BENCH INFRASTRUCTURE, not product).

Times the reference's per-partition work restated by the oracle: for every
point ``np.linalg.norm(C - x, axis=1)`` + ``np.argmin`` (kmeans_spark.py:147-159)
and the map-side combine of ``reduceByKey`` (kmeans_spark.py:169-171), one
worker process per partition like Spark ``local[N]``.  PySpark/JVM overheads
(pickling, shuffle, scheduling) are not included, so this is an optimistic
CPU number.
"""
from __future__ import annotations

import time

import numpy as np


def _sample(d, k, n, seed):
    rng = np.random.default_rng(seed)
    centers = rng.uniform(-10, 10, (k, d))
    X = centers[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    C = X[rng.choice(n, k, replace=False)] if n >= k else centers
    return X, C


def _assign(part, C):
    for point in part:
        dist = np.linalg.norm(C - point, axis=1)      # L153
        yield int(np.argmin(dist)), (point, 1)        # L156-159


def _merge(a, b):                                     # reduceByKey lambda, L169-171
    return a[0] + b[0], a[1] + b[1]


def _partition_pass(X, C):
    # map-side combine of reduceByKey over the streamed (cid, (point, 1)) pairs
    acc = {}
    for cid, val in _assign(X, C):
        acc[cid] = _merge(acc[cid], val) if cid in acc else val
    return acc


def _cached_rows(X):
    # a cached partition holds its rows as Python objects (rdd.cache(), L256):
    # the per-point views exist before the pass, as in the PySpark stand-in
    return list(X)


def calibrate(d, k, n=2000):
    X, C = _sample(d, k, n, 0)
    rows = _cached_rows(X)
    t0 = time.perf_counter()
    _partition_pass(rows, C)
    return n / (time.perf_counter() - t0)


def run_partition(d, k, n, seed, start_at=None):
    """One partition's pass; returns (points, pass start, pass end) on the
    system-wide monotonic clock (time.monotonic, shared by the worker
    processes), so the caller times only the passes, not the workers'
    start-up, imports or data generation.  ``start_at``: wait until that
    monotonic time, so every worker's pass starts together."""
    X, C = _sample(d, k, n, seed + 1)
    rows = _cached_rows(X)
    if start_at is not None:
        while time.monotonic() < start_at:
            time.sleep(min(0.01, max(0.0, start_at - time.monotonic())))
    t0 = time.monotonic()
    _partition_pass(rows, C)
    return n, t0, time.monotonic()
