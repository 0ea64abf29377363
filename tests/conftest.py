import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)


# KM_LIB=diag: run against the diagnostic library (libkmeans_amd_diag.so,
# `make -C <pkg>/csrc diag`), which adds the fast-screen experiment
# (km_set_screen modes 2 and 3) to the product kernels
DIAG_LIB = os.environ.get("KM_LIB") == "diag"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    if DIAG_LIB:
        sys.path.insert(0, ROOT)
        from kmeans_amd import _lib
        _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), "libkmeans_amd_diag.so")


def load_golden(name):
    """Fixture dict (+ regenerated X when it is not stored)."""
    import make_golden  # tests/golden/make_golden.py (no reference import at module load)
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    out = {key: z[key] for key in z.files}
    if "X" in out:
        X = out["X"].astype(np.float64)
    else:
        X = make_golden.case_data(make_golden.CASES[name]["data"])
    assert make_golden.x_digest(X) == str(out["x_sha256"]), f"{name}: regenerated data drifted"
    out["X"] = X
    out["stdout"] = str(out["stdout"])
    return out


GOLDEN_CASES = ["test_a", "test_c", "test_d", "test_e_p3", "test_b_small", "empty", "ties",
                "c2_small", "c3_small", "c4_small", "tight", "tight_wide", "c5_poor", "c1"]
# float32 rows given to the reference as float32 (it then computes in float32
# throughout: kmeans_spark.py:153, 176, 184, 231-233); the product computes in
# float64 on the same rows, held to the north-star bars
F32_CASES = ["f32_test_a", "f32_c1", "f32_c3_small", "f32_empty"]


def check_float32_run(g, centroids, sse_history, labels, log_text):
    """North-star bars against a reference run on float32 rows.

    centroids: the reference returns the input dtype (zeros_like,
    kmeans_spark.py:176), so float32 here too, within 1e-5 of the data scale.
    SSE: the reference adds float32 min_distance ** 2 terms into a float32
    partition_sse (Python float + np.float32 is np.float32 under NumPy 2,
    :229-233), so its own error is up to m * 2^-24 relative for m rows per
    partition (plus the partition .sum()); the bar is that bound, at least
    1e-6.  Labels: equal except where the reference centroids' float64 top-2
    distances are within 1e-6 relative plus twice the largest centroid
    difference (triangle inequality: a point can only change sides by that
    much).  Log lines: same lines, numbers within 1e-5 relative."""
    ref_c = g["centroids"]
    assert centroids.dtype == np.float32, centroids.dtype
    scale = float(np.abs(g["X"]).max())
    np.testing.assert_allclose(centroids, ref_c, rtol=1e-5, atol=1e-5 * scale)
    n, slices = int(g["n"]), int(g["slices"])
    m = -(-n // slices)
    rtol_sse = max(1e-6, (m + slices) * 2.0 ** -24)
    assert len(sse_history) == len(g["sse_history"])
    np.testing.assert_allclose(sse_history, g["sse_history"], rtol=rtol_sse)
    X = g["X"]
    D = np.sqrt(((X[:, None, :] - ref_c[None].astype(np.float64)) ** 2).sum(-1)) if len(ref_c) * len(X) <= 4e7 \
        else None
    bad = np.nonzero(labels != g["labels"])[0]
    if len(bad):
        assert D is not None, "label mismatch on a case too large for the band check"
        e = float(np.sqrt(((centroids.astype(np.float64) - ref_c) ** 2).sum(-1)).max())
        dp, dr = D[bad, labels[bad]], D[bad, g["labels"][bad]]
        assert np.all(dp - dr <= 1e-6 * dr + 2 * e), (bad[:10], (dp - dr)[:10], e)
        assert len(bad) <= max(2, len(X) // 1000), len(bad)
    import re
    num = re.compile(r"[-+]?\d+\.\d+")
    a = [ln for ln in log_text.splitlines() if ln.strip()]
    b = [ln for ln in g["stdout"].splitlines() if ln.strip()]
    assert len(a) == len(b), (a, b)
    for x, y in zip(a, b):
        assert num.sub("#", x) == num.sub("#", y), (x, y)
        for u, v in zip(num.findall(x), num.findall(y)):
            assert abs(float(u) - float(v)) <= 1e-5 * abs(float(v)) + 2 * 10 ** -len(v.split(".")[1]), (x, y)


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]
    return get
