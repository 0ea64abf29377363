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
