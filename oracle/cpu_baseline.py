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


def _partition_pass(X, C):
    acc = {}
    for point in X:
        dist = np.linalg.norm(C - point, axis=1)      # L153
        cid = int(np.argmin(dist))                    # L156
        if cid in acc:                                # reduceByKey lambda, L169-171
            s, c = acc[cid]
            acc[cid] = (s + point, c + 1)
        else:
            acc[cid] = (point, 1)
    return acc


def calibrate(d, k, n=2000):
    X, C = _sample(d, k, n, 0)
    t0 = time.perf_counter()
    _partition_pass(X, C)
    return n / (time.perf_counter() - t0)


def run_partition(d, k, n, seed):
    X, C = _sample(d, k, n, seed + 1)
    t0 = time.perf_counter()
    _partition_pass(X, C)
    return n, time.perf_counter() - t0
