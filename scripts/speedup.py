"""Speedup sweep tooling: the counterpart of the reference's test_e
(kmeans_spark.py:543-621, "Speedup vs Number of Partitions").

    python scripts/speedup.py table FILE [FILE ...] [--png speedup_graph.png]
        Bench lines of ``bench.py --gpus N`` (one JSON object per line, or the
        driver's SCALE_rNN.json holding them) -> the reference's timing table
        (time per step, speedup vs the smallest N, scaling efficiency) and the
        ideal-vs-actual speedup figure.  Strong scaling (fixed N rows, the
        metric's configuration): speedup = value(N) / value(N_min).

    python scripts/speedup.py partitions [--png speedup_graph.png]
        test_e's own workload on this GPU: make_blobs-style 50,000 x 10,
        k=5, max_iter=10, fit timed for 1..4 partitions of the input (the
        reference's partitions are Spark tasks; here they only change the
        takeSample layout, the GPU does the same work), same table + figure.

The table lines are the reference's (``Partitions: n | Time: t s | Speedup: s x``,
kmeans_spark.py:591-592), with GPUs in place of partitions for ``table``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_objects(obj):
    """Every bench line (a dict with n_gpus and value) inside a JSON value."""
    if isinstance(obj, dict):
        if "n_gpus" in obj and "value" in obj:
            yield obj
        for v in obj.values():
            yield from _bench_objects(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from _bench_objects(v)
    elif isinstance(obj, str) and '"n_gpus"' in obj:
        for line in obj.splitlines():
            line = line.strip()
            if line.startswith("{"):
                try:
                    yield from _bench_objects(json.loads(line))
                except ValueError:
                    pass


def load_runs(paths):
    runs = {}
    for p in paths:
        text = open(p).read()
        try:
            objs = list(_bench_objects(json.loads(text)))
        except ValueError:
            objs = list(_bench_objects(text))
        for o in objs:
            runs[int(o["n_gpus"])] = o   # the last line per N wins
    if not runs:
        raise SystemExit("no bench lines (objects with n_gpus and value) found")
    return dict(sorted(runs.items()))


def speedup_table(runs):
    """[(n, seconds per step, speedup, efficiency)] relative to the smallest n."""
    n0 = min(runs)
    base = runs[n0]["value"]
    rows = []
    for n, o in runs.items():
        sec = (o.get("ms_per_step") or 1e3 / o["value"]) / 1e3
        s = o["value"] / base
        rows.append((n, sec, s, s / (n / n0)))
    return rows


def print_table(rows, unit="GPUs"):
    print("\n[Timing Summary]")
    for n, sec, s, eff in rows:
        print(f"{unit}: {n:2d} | Time: {sec:8.4f}s | Speedup: {s:6.4f}x | Efficiency: {eff:6.1%}")


def plot(rows, path, xlabel):
    try:
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        print("matplotlib not available: figure skipped")
        return None
    n = np.array([r[0] for r in rows])
    s = np.array([r[2] for r in rows])
    plt.figure(figsize=(10, 6))
    plt.plot(n, n / n[0], "b-", marker="o", linewidth=2, markersize=8, label="Ideal")
    plt.plot(n, s, "orange", marker="s", linewidth=2, markersize=8, label="Actual")
    plt.xlabel(xlabel, fontsize=12)
    plt.ylabel("Speedup", fontsize=12)
    plt.title(f"Speedup vs {xlabel}", fontsize=14, fontweight="bold")
    plt.legend(fontsize=11)
    plt.grid(True, alpha=0.3)
    plt.xticks(list(n))
    plt.savefig(path, dpi=150, bbox_inches="tight")
    plt.close()
    print(f"Graph saved to: {path}")
    return path


def run_partitions(counts=(1, 2, 3, 4), n=50_000, d=10, k=5, max_iter=10, seed=42):
    """test_e's workload through this package's KMeans on the local GPU."""
    sys.path.insert(0, ROOT)
    import kmeans_amd as ka
    rng = np.random.default_rng(seed)
    centers = rng.uniform(-10, 10, (5, d))
    X = centers[rng.integers(0, 5, n)] + rng.standard_normal((n, d))
    print(f"\nDataset: {X.shape[0]} points, {X.shape[1]} dimensions")
    print(f"K-Means Parameters: k={k}, max_iter={max_iter}")
    sc = ka.LocalContext()
    warm = ka.KMeans(k=k, max_iter=1, seed=seed)   # untimed: HIP context and module start-up
    warm.verbose = False
    warm.fit(sc.parallelize(X[:1000], 1), sc)
    times = {}
    for p in counts:
        rdd = sc.parallelize(X, numPartitions=p).cache()
        km = ka.KMeans(k=k, max_iter=max_iter, tolerance=1e-4, seed=seed, compute_sse=False)
        km.verbose = False
        t0 = time.time()
        km.fit(rdd, sc)
        times[p] = time.time() - t0
        print(f"\nPartitions: {p}\nTime: {times[p]:.4f} seconds")
    base = times[counts[0]]
    return [(p, times[p], base / times[p], base / times[p] / p) for p in counts]


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("table")
    t.add_argument("files", nargs="+")
    t.add_argument("--png", default=None)
    p = sub.add_parser("partitions")
    p.add_argument("--png", default=None)
    args = ap.parse_args()
    if args.cmd == "table":
        rows = speedup_table(load_runs(args.files))
        print_table(rows)
        if args.png:
            plot(rows, args.png, "Number of GPUs")
    else:
        rows = run_partitions()
        print_table(rows, unit="Partitions")
        if args.png:
            plot(rows, args.png, "Number of Partitions")


if __name__ == "__main__":
    main()
