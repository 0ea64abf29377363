"""c2 small path: assign kernel with fused float64 statistics (Lloyd step) vs
the same kernel without them (predict), HIP-event averages.  Shows how much of
k_assign_small is the LDS statistics table.
Usage: python scripts/small_probe.py [config] [N] [--diag]   (--diag: load the
diagnostic library, libkmeans_amd_diag.so, whose KM_* environment knobs apply)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (CONFIGS, package alias)
import kmeans_amd  # noqa: E402
if "--diag" in sys.argv:
    sys.argv.remove("--diag")
    kmeans_amd._lib.LIB_PATH = kmeans_amd._lib.LIB_PATH.replace("libkmeans_amd.so", "libkmeans_amd_diag.so")
from kmeans_amd.comm import Communicator  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
N, d, k, centers = bench.CONFIGS[cfg]
if len(sys.argv) > 2:                         # row count override (steady state vs launch ramp)
    N = int(sys.argv[2])
km = kmeans_amd.KMeans(k=k, max_iter=10 ** 9, tolerance=1e-300, seed=42, compute_sse=False)
km.verbose = False
data = kmeans_amd.DeviceBlobs(n=N, d=d, n_centers=centers, box=10.0, std=1.0, seed=2024)
run = km._make_runner(data, Communicator())
eng = run.engine
eng.set_centroids(km._initialize_centroids(run))
for i in range(3):
    run.iteration(km, i, None)
eng.sync()
eng.profile(True, phases=("assign",))
for i in range(20):
    run.iteration(km, 3 + i, None)
eng.sync()
ms_fit, n_fit = eng.prof_read("assign")
eng.profile(True, phases=("assign",))
for i in range(20):
    eng.predict()
eng.sync()
ms_pred, n_pred = eng.prof_read("assign")
eng.profile(False)
ms_fit, ms_pred = ms_fit / max(n_fit, 1), ms_pred / max(n_pred, 1)  # prof_read: total ms, launches
gb = N * d * 4 / 1e9
print(f"{cfg}: assign+stats {ms_fit * 1e3:.1f} us ({gb / ms_fit * 1e3:.0f} GB/s, {n_fit} launches); "
      f"assign only {ms_pred * 1e3:.1f} us ({gb / ms_pred * 1e3:.0f} GB/s, {n_pred} launches)")
