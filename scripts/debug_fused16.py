"""Debug aid for the fused screen (tests/test_gpu_fast_screen.py cases): fit one
step with a forced screen and predict, report mismatches against the oracle
with the distances of the chosen and the true centroid.
usage: python scripts/debug_fused16.py [case] [screen]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import kmeans_oracle as orc  # noqa: E402
from test_gpu_fast_screen import _blobs, _fit  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "far"
mode = int(sys.argv[2]) if len(sys.argv) > 2 else 0
if case == "far":
    X = _blobs(20000, 64, 128, seed=5, box=1000.0, std=1.0)
    C0 = X[np.random.default_rng(2).choice(len(X), 256, replace=False)]
else:
    X = _blobs(60000, 64, 256, seed=3)
    C0 = X[np.random.default_rng(1).choice(len(X), 256, replace=False)]


def report(what, got, C):
    want = orc.assign(X, C)[0]
    bad = np.nonzero(got != want)[0]
    print(f"{what}: {len(bad)} mismatches of {len(X)}")
    for r in bad[:12]:
        D = np.linalg.norm(C - X[r], axis=1)
        order = np.argsort(D)
        print(f"  row {r}: got {got[r]} (D {D[got[r]]:.6f}, rank {int(np.nonzero(order == got[r])[0][0])}) "
              f"want {want[r]} (D {D[want[r]]:.6f}); chains got {got[r] & 15} want {want[r] & 15}; "
              f"row%32 {r % 32}")
    if len(bad):
        print("  rows mod 32 histogram:", np.bincount(bad % 32, minlength=32).tolist())
    return len(bad)


km = _fit(X, C0, mode)
report(f"fit labels (screen {mode})", km._runner.engine.labels(), C0)
C1 = km.centroids
report("predict (REF)", km.predict(X).to_numpy(), C1)
km2 = _fit(X, C1, mode)
report(f"fit from the fitted centroids (screen {mode})", km2._runner.engine.labels(), C1)
km3 = _fit(X, C1, 1)
report("fit from the fitted centroids (screen 1, REF)", km3._runner.engine.labels(), C1)
