"""Pins the resolvers against floating-point contraction (exactness).

hipcc contracts ``acc + t * t`` into ``v_fma_f64`` unless a
``#pragma clang fp contract(off)`` covers the add (checked on this toolchain
with the product flags: plain kernel code and a new helper without the pragma
get ``v_fma_f64``; the helpers of csrc/km_exact.h get ``v_mul_f64`` + add).
An fma skips the rounding of the square, so a contracted pairwise sum is not
``np.linalg.norm`` (kmeans_spark.py:153).  That is how a round-1 scan variant
"computed wrong norms inside the kernel" while the km_exact.h helpers were
exact in the probe.

The cases below are near-tie pairs (x, c1, c2) where the contracted sum picks
the OTHER centroid than NumPy does (fma emulated exactly with fractions), so
any contraction reaching a resolver flips their labels.  Each case sits in its
own region of space, so only its own pair (or triple) competes.  Checked on
the small path (in-thread re-rank), the MFMA path's re-rank (k_rerank2, pairs)
and its full scan (k_fullscan, triples).
"""
from fractions import Fraction

import numpy as np
import pytest

from oracle import kmeans_oracle as orc

pytestmark = pytest.mark.gpu

D = 16


def _np_sum(c, x):
    t = c - x.astype(np.float64)
    return float(np.add.reduce(t * t))      # NumPy's pairwise order for d = 16


def _fma_sum(c, x):
    # NumPy's 8-accumulator order for 8 <= d <= 128, with the second-round
    # squares fused into their accumulators (what contraction produces)
    t = [float(ci - float(xi)) for ci, xi in zip(c, x)]
    r = [ti * ti for ti in t[:8]]
    for i in range(8, len(t)):
        r[i % 8] = float(Fraction(t[i]) * Fraction(t[i]) + Fraction(r[i % 8]))   # fma, rounded once
    return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))


def _argmin(sums):
    return int(np.argmin(sums))               # np.argmin: first index on ties


def _cases(m, triple, seed):
    """Rows and centroids of m near-tie cases whose NumPy and contracted
    picks differ.  Case i lives at 1000 (i + 1) along feature 0 (only its own
    centroids compete); its centroids are c1 and c2 = c1 nudged by a few ulps
    in one second-round feature (plus c2's next double up for triples)."""
    rng = np.random.default_rng(seed)
    X, C = [], []
    while len(X) < m:
        sh = np.zeros(D)
        sh[0] = 1000.0 * (len(X) + 1)
        x = (rng.uniform(-1, 1, D) + sh).astype(np.float32)
        c1 = x.astype(np.float64) + rng.normal(0, 0.3, D)
        c2 = c1.copy()
        f = rng.integers(8, D)
        for _ in range(rng.integers(1, 6)):
            c2[f] = np.nextafter(c2[f], np.inf if rng.random() < 0.5 else -np.inf)
        cs = [c1, c2] + ([np.nextafter(c2, np.inf)] if triple else [])
        npy = [_np_sum(c, x) for c in cs]
        fma = [_fma_sum(c, x) for c in cs]
        if _argmin(npy) != _argmin(fma) and len(set(np.sqrt(npy))) == len(cs):
            X.append(x)
            C += cs
    return np.array(X, dtype=np.float64), np.array(C)


def _labels(X, C):
    import kmeans_amd as ka

    class Pinned(ka.KMeans):
        def _initialize_centroids(self, run):
            return C.copy()

    km = Pinned(k=len(C), max_iter=1, tolerance=1e-12)
    km.verbose = False
    km.fit(X)
    return km._runner.engine.labels()


@pytest.mark.parametrize("m,triple,path", [(12, False, "small (k <= 32)"), (40, False, "MFMA + k_rerank2"),
                                           (30, True, "MFMA + k_fullscan")])
def test_resolvers_are_not_contracted(m, triple, path):
    X, C = _cases(m, triple, seed=m + 7 * triple)
    want = orc.assign(X, C)[0]
    s = 3 if triple else 2
    assert np.array_equal(want // s, np.arange(m))          # only a case's own centroids compete
    got = _labels(X, C)
    np.testing.assert_array_equal(got, want, err_msg=path)
