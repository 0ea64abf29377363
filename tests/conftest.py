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
                "c2_small", "c3_small", "c4_small", "tight", "tight_wide", "c5_poor"]


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]
    return get
