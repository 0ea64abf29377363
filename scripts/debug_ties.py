"""Diagnostic (GPU box): near-tie labels vs the oracle, per path."""
import os, sys, json
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import kmeans_oracle as orc
import kmeans_amd as ka


def blobs(n, d, centers, seed):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-10, 10, (centers, d))
    X = C[rng.integers(0, centers, n)] + rng.standard_normal((n, d))
    return X.astype(np.float32).astype(np.float64)


n, d, nb = [int(v) for v in sys.argv[1:4]]
X = blobs(n, d, 64, 11 + d)
rng = np.random.default_rng(5 + d)
base = X[rng.choice(len(X), nb, replace=False)]
C0 = np.concatenate([base, np.nextafter(base, np.inf)])


class Pinned(ka.KMeans):
    def _initialize_centroids(self, run):
        return C0.copy()


km = Pinned(k=len(C0), max_iter=1, tolerance=1e-12, compute_sse=True)
km.verbose = False
km.fit(X)
lab = km._runner.engine.labels()
ref = orc.assign(X, C0)[0]
D = orc.distances(X, C0)
bad = np.nonzero(lab != ref)[0]
print(json.dumps({"fused": os.environ.get("KM_FUSED", "1"), "bad": len(bad), "last": {k: v for k, v in km._runner.last.items() if k != "counts"}}))
for i in bad[:8]:
    a, b = int(lab[i]), int(ref[i])
    print(i, "gpu", a, "ref", b, repr(D[i, a]), repr(D[i, b]), "row_is_base", bool((X[i] == base).all(1).any()))
