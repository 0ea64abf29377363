"""Stream-time cost of the bench's per-launch HIP events: the same Lloyd
iterations timed with and without events around the dominant kernel,
alternating on one engine.  usage: python scripts/probes/prof_overhead.py [config] [steps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import kmeans_amd  # noqa: E402
from kmeans_amd.comm import Communicator  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
N, d, k, centers = bench.CONFIGS[cfg]
km = kmeans_amd.KMeans(k=k, max_iter=10 ** 9, tolerance=1e-300, seed=42, compute_sse=False)
km.verbose = False
data = kmeans_amd.DeviceBlobs(n=N, d=d, n_centers=centers, box=10.0, std=1.0, seed=2024)
run = km._make_runner(data, Communicator())
eng = run.engine
eng.set_centroids(km._initialize_centroids(run))
km.sse_history = []
done = 3
run.run(km, None, done)
eng.sync()
res = {"events": [], "none": []}
for rnd in range(4):
    for mode in ("events", "none"):
        eng.profile(mode == "events", phases=("assign", "stats"))
        t0 = time.perf_counter()
        run.run(km, None, done + steps, first=done)
        eng.sync()
        t1 = time.perf_counter()
        done += steps
        res[mode].append((t1 - t0) / steps * 1e6)
eng.profile(False)
for mode, v in res.items():
    print(f"{cfg} {mode}: us/step {np.round(v, 1).tolist()} median {np.median(v):.1f}")
