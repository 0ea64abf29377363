"""Lockstep full-scan forensics (GPU box): labels of the c3-shape one-step case
against the oracle; for the mismatched rows, what the kernel chose."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import kmeans_amd as ka
from oracle import kmeans_oracle as orc

n, d, k, centers = 50000, 64, 256, 256
rng = np.random.default_rng(n + d + k)
Cb = rng.uniform(-10, 10, (centers, d))
lab = rng.integers(0, centers, n)
X = (Cb[lab] + rng.standard_normal((n, d))).astype(np.float32).astype(np.float64)
C0 = X[np.random.default_rng(1).choice(n, k, replace=False)]


class Pinned(ka.KMeans):
    def _initialize_centroids(self, run):
        return C0.copy()


km = Pinned(k=k, max_iter=1, tolerance=1e-12, compute_sse=True)
km.verbose = False
km.fit(X)
got = km._runner.engine.labels()
ref, dist, gap = orc.assign(X, C0)
bad = np.nonzero(got != ref)[0]
print("mismatches", len(bad), "q_rerank", km._runner.last["q_rerank"], "q_full", km._runner.last["q_full"])
D = np.sqrt(((X[bad, None, :] - C0[None]) ** 2).sum(-1)) if len(bad) else None
for i, r in enumerate(bad[:25]):
    order = np.argsort(D[i], kind="stable")[:4]
    print(r, "got", got[r], "ref", ref[r], "top4", order.tolist(), np.round(D[i][order], 4).tolist(),
          "d(got)", round(float(D[i][got[r]]), 4))
