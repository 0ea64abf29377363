"""Pin the CPU oracle (oracle/kmeans_oracle.py) against golden vectors that
tests/golden/make_golden.py produced by running the reference KMeans itself
(kmeans_spark.py:239-352 under the PySpark stand-in)."""
import numpy as np
import pytest

from conftest import GOLDEN_CASES
from oracle import kmeans_oracle as orc


def _fit(g, faithful=False):
    lines = []
    res = orc.lloyd_fit(g["X"], int(g["k"]), int(g["max_iter"]), float(g["tol"]), int(g["seed"]),
                        bool(g["sse"]), int(g["slices"]), init_centroids=g["init"],
                        empty_seed=lambda: int(g["time_seed"]), log=lines.append, faithful=faithful)
    return res, lines


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_reference_bitwise(golden, name):
    g = golden(name)
    res, lines = _fit(g)
    # centroids and SSE are bit-identical: same expressions, same reduction order
    np.testing.assert_array_equal(res["centroids"], g["centroids"])
    np.testing.assert_array_equal(np.asarray(res["sse_history"]), g["sse_history"])
    # the log stream (kmeans_spark.py:192,262-263,285,299-303,311) is identical
    assert "\n".join(lines) + "\n" == g["stdout"]
    np.testing.assert_array_equal(orc.predict(g["X"], res["centroids"]), g["labels"])


@pytest.mark.parametrize("name", ["test_a", "test_d", "ties", "empty"])
def test_oracle_takesample_init_matches_reference(golden, name):
    g = golden(name)
    if name in ("ties", "empty"):
        pytest.skip("case injects its initial centroids")
    sizes = [b - a for a, b in orc.partition_bounds(int(g["n"]), int(g["slices"]))]
    idx = orc.take_sample_indices(sizes, int(g["k"]), int(g["seed"]))
    np.testing.assert_array_equal(g["X"][idx], g["init"])


@pytest.mark.parametrize("name", ["test_a", "ties"])
def test_faithful_and_vectorised_agree(golden, name):
    g = golden(name)
    a, _ = _fit(g, faithful=True)
    b, _ = _fit(g, faithful=False)
    np.testing.assert_array_equal(a["centroids"], b["centroids"])
    np.testing.assert_array_equal(np.asarray(a["sse_history"]), np.asarray(b["sse_history"]))


def test_vectorised_distance_bitwise_equals_linalg_norm():
    rng = np.random.default_rng(0)
    X = rng.standard_normal((257, 37))
    C = rng.standard_normal((11, 37)) * 3
    D = orc.distances(X, C, chunk=64)
    for i in range(0, 257, 17):
        np.testing.assert_array_equal(D[i], np.linalg.norm(C - X[i], axis=1))


def test_oracle_validation_messages():
    X = np.zeros((4, 2))
    with pytest.raises(ValueError, match="k must be positive, got 0"):
        orc.lloyd_fit(X, 0)
    with pytest.raises(ValueError, match="max_iter must be positive, got 0"):
        orc.lloyd_fit(X, 2, max_iter=0)
    with pytest.raises(ValueError, match="tolerance must be positive, got 0"):
        orc.lloyd_fit(X, 2, tolerance=0)
    with pytest.raises(ValueError, match=r"Not enough data points \(4\) to initialize 5 clusters"):
        orc.lloyd_fit(X, 5)


def _np_order_norm(c, x):
    """The summation order the HIP resolvers implement (km_kernels.hip np_norm):
    rounded (c - x)^2 terms, NumPy pairwise_sum blocks of <= 128 with 8
    strided accumulators, halves split at n/2 rounded down to a multiple of 8."""
    t = [(float(cf) - float(xf)) * (float(cf) - float(xf)) for cf, xf in zip(c, x)]

    def block(a):
        if len(a) < 8:
            r = 0.0
            for v in a:
                r += v
            return r
        r = list(a[:8])
        nm = len(a) - len(a) % 8
        for i in range(8, nm, 8):
            for u in range(8):
                r[u] += a[i + u]
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
        for v in a[nm:]:
            res += v
        return res

    def pw(a):
        if len(a) <= 128:
            return block(a)
        n2 = len(a) // 2
        n2 -= n2 % 8
        return pw(a[:n2]) + pw(a[n2:])

    return np.sqrt(pw(t))


@pytest.mark.parametrize("d", [1, 2, 7, 8, 9, 15, 16, 17, 64, 100, 127, 128, 129, 136, 200, 250, 255, 256])
def test_resolver_summation_order_is_linalg_norm(d):
    # near-tie centroids (one float64 ulp apart) make any other order show
    rng = np.random.default_rng(d)
    X = (rng.standard_normal((40, d)) * 5).astype(np.float32).astype(np.float64)
    base = rng.standard_normal((6, d)) * 5
    C = np.concatenate([base, np.nextafter(base, np.inf), np.nextafter(base, -np.inf)])
    for x in X:
        ref = np.linalg.norm(C - x, axis=1)
        got = np.array([_np_order_norm(c, x) for c in C])
        np.testing.assert_array_equal(got, ref)
