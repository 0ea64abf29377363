"""Cross-check of bench.py's CPU baseline against the reference itself.

bench.py's ``cpu_baseline`` leg times ``oracle/cpu_baseline.py``, a restatement
of the reference's map-side work (per point ``np.linalg.norm(C - x, axis=1)`` +
``np.argmin``, kmeans_spark.py:147-159, and the reduceByKey combine,
kmeans_spark.py:169-171).  This script times, on one core and on the same
(X, C), that restatement against the reference's own closures: the reference
module imported unmodified with the in-memory PySpark stand-in
(tests/golden/_pyspark_stub, as tests/golden/make_golden.py does), running
its per-point work over one partition: ``KMeans._assign_to_clusters`` and
the ``reduceByKey`` with the reference's own combine lambda (captured from
``KMeans._update_centroids`` through a recording proxy, kmeans_spark.py:169-171).
The driver-side rest of ``_update_centroids`` (a Python loop over the k
clusters per iteration) is not per-point work and is left out, as the
oracle's extrapolation to N leaves it out.  The two sides run as adjacent pairs (reference, then oracle, on
the same sample), repeated; the verdict is the MEDIAN of the per-pair
throughput ratios, which cancels the slow drift of a shared VM's speed (+-15 %
between runs here) and ignores outliers.  Both are pinned to one core, timed
in process CPU time (time.process_time, not inflated by VM steal), with the
garbage collector paused in the timed regions (the stand-in materialises
every yielded tuple, which real Spark streams into the combiner).  It asserts the two throughputs agree within
10 %.

Runs in the development container only (it reads /root/reference, which does
not exist on the GPU box):

    python scripts/check_cpu_baseline.py [--scale 1.0] [--reps 0] [--tol 0.10]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

SHAPES = [  # (name, d, k, points per repetition, repetitions): the BASELINE.json configs' row shapes
    ("c2", 16, 8, 10000, 21),
    ("c3", 64, 256, 5000, 21),
    ("c4", 32, 1024, 2500, 21),
    ("c5", 128, 4096, 800, 9),
]


class _Captured(Exception):
    pass


class _RecordingRDD:
    """Stands in for the assigned RDD to learn the function
    ``_update_centroids`` passes to ``reduceByKey`` (L169-171)."""

    def reduceByKey(self, f):
        self.f = f
        raise _Captured


def reference_combine(ref, sc, C):
    km = ref.KMeans(k=len(C), max_iter=1, tolerance=1e-4, seed=42, compute_sse=False)
    km.centroids = C.copy()
    rec = _RecordingRDD()
    try:
        km._update_centroids(rec, None, sc, sc.broadcast(C))
    except _Captured:
        return rec.f
    raise RuntimeError("reduceByKey was not reached")


def time_reference(ref, X, C, reps):
    sc = ref.SparkContext(appName="cpu-baseline-check")
    rdd = sc.parallelize(X, 1)
    combine = reference_combine(ref, sc, C)
    best = float("inf")
    for _ in range(reps):
        km = ref.KMeans(k=len(C), max_iter=1, tolerance=1e-4, seed=42, compute_sse=False)
        km.centroids = C.copy()
        bc = sc.broadcast(C)
        t0 = time.process_time()
        assigned = km._assign_to_clusters(rdd, bc)             # L147-161 (eager in the stand-in)
        assigned.reduceByKey(combine)                          # L169-171, the reference's lambda
        best = min(best, time.process_time() - t0)
    return len(X) / best


def time_oracle(cb, X, C, reps):
    X = cb._cached_rows(X)
    best = float("inf")
    for _ in range(reps):
        t0 = time.process_time()
        cb._partition_pass(X, C)
        best = min(best, time.process_time() - t0)
    return len(X) / best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0, help="multiply the per-shape point counts")
    ap.add_argument("--reps", type=int, default=0, help="pairs per shape (0: the table's)")
    ap.add_argument("--tol", type=float, default=0.10)
    args = ap.parse_args()
    import contextlib
    import io

    import gc

    import cpu_baseline as cb
    from make_golden import import_reference
    if hasattr(os, "sched_setaffinity"):
        os.sched_setaffinity(0, {sorted(os.sched_getaffinity(0))[-1]})
    try:
        # c5's per-point temporaries (C - x: 4 MiB) would be mapped and
        # unmapped by glibc on every call; keep them on the heap so page-fault
        # noise does not dominate either side
        import ctypes
        libc = ctypes.CDLL("libc.so.6")
        libc.mallopt(-3, 256 << 20)   # M_MMAP_THRESHOLD
        libc.mallopt(-1, 512 << 20)   # M_TRIM_THRESHOLD
    except OSError:
        pass
    ref = import_reference()
    ok = True
    for name, d, k, n, reps in SHAPES:
        n = max(2, int(n * args.scale))
        X, C = cb._sample(d, k, n, 7)
        ratios, refs, orcs = [], [], []
        for _ in range(reps if args.reps <= 0 else args.reps):
            gc.collect()
            gc.disable()
            with contextlib.redirect_stdout(io.StringIO()):   # the reference logs empty-cluster repairs
                refs.append(time_reference(ref, X, C, 1))
            gc.enable()
            gc.collect()
            gc.disable()
            orcs.append(time_oracle(cb, X, C, 1))
            gc.enable()
            ratios.append(orcs[-1] / refs[-1])
        ratio = float(np.median(ratios))
        r_ref, r_orc = float(np.median(refs)), float(np.median(orcs))
        good = abs(ratio - 1.0) <= args.tol
        ok &= good
        print(f"{name}: d={d} k={k} n={n} x {len(ratios)} pairs  reference {r_ref:,.0f} pts/s  oracle {r_orc:,.0f} "
              f"pts/s (medians)  median pair ratio {ratio:.3f} [{min(ratios):.2f}..{max(ratios):.2f}]  "
              f"{'ok' if good else 'OUT OF TOLERANCE'}")
    if not ok:
        sys.exit(1)


if __name__ == "__main__":
    main()
