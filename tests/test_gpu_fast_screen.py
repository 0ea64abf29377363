"""Every screen of the fused kernel returns the reference's labels.

The fused path (k_fused, the c3 class: k <= 256, d <= 64) has two screens in
the product library (km_set_screen): fp16x3 with the global bound and fp16x3
with per-key bounds.  The diagnostic library (KM_LIB=diag) adds the fast
screen (k_fused1: one fp16 MFMA per product against a balanced fp16 image,
PAIRWISE bound; row as one fp16 part, or hi + lo), which lost end to end on
every BASELINE shape and is not in the product build.  The choice is a cost
choice, so each mode is forced here and held to the same bar as the automatic
choice: labels equal to
np.argmin(np.linalg.norm(C - x, axis=1)) (kmeans_spark.py:153-156) bit for
bit, centroids and SSE at 1e-9 against the oracle (kmeans_spark.py:147-237).

The cases aim at the fast screen's decision band: one-ulp duplicate
centroids, points placed on and near bisector planes of close centroid pairs
at distances from 1e-7 to 1 (the pairwise bound is ~1e-2 of the distances
here), far-from-origin clusters (||c|| ||x|| >> distances), rows whose
features span 12 orders of magnitude (fp16 subnormals after scaling), and a
multi-iteration fit on noise (test_b style).
"""
import numpy as np
import pytest

from oracle import kmeans_oracle as orc

from conftest import DIAG_LIB

pytestmark = pytest.mark.gpu

MODES = [0, 1, 2, 3] if DIAG_LIB else [0, 1]
diag_only = pytest.mark.skipif(not DIAG_LIB, reason="fast screen: diagnostic library only (KM_LIB=diag)")


def _km():
    import kmeans_amd
    return kmeans_amd


def _fit(X, C0, mode, iters=1, compute_sse=True):
    ka = _km()
    from kmeans_amd.engine import make_engine

    def factory(comm):
        eng = make_engine(comm)
        eng.set_screen(mode)
        return eng

    class Forced(ka.KMeans):
        _engine_factory = staticmethod(factory)

        def _initialize_centroids(self, run):
            return C0.copy()

    km = Forced(k=len(C0), max_iter=iters, tolerance=1e-12, compute_sse=compute_sse)
    km.verbose = False
    km.fit(X)
    return km


def _check(X, C0, mode, iters=1):
    km = _fit(X, C0, mode, iters)
    ref = orc.lloyd_fit(X, len(C0), iters, 1e-12, 0, True, 1, init_centroids=C0)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
    # labels of the last fit pass (against the centroids that pass used)
    C_last = C0 if iters == 1 else orc.lloyd_fit(X, len(C0), iters - 1, 1e-12, 0, True, 1,
                                                  init_centroids=C0)["centroids"]
    np.testing.assert_array_equal(km._runner.engine.labels(), orc.assign(X, C_last)[0])
    # predict with the final centroids (same screen)
    np.testing.assert_array_equal(km.predict(X).to_numpy(), orc.assign(X, ref["centroids"])[0])
    return km


def _blobs(n, d, centers, seed, box=10.0, std=1.0):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-box, box, (centers, d))
    lab = rng.integers(0, centers, n)
    return (C[lab] + std * rng.standard_normal((n, d))).astype(np.float32).astype(np.float64)


@pytest.mark.parametrize("mode", MODES)
def test_c3_shape_one_step(mode):
    X = _blobs(60000, 64, 256, seed=3)
    C0 = X[np.random.default_rng(1).choice(len(X), 256, replace=False)]
    _check(X, C0, mode)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("nb", [128, 127])
def test_one_ulp_duplicates(mode, nb):
    # duplicates on the same chain (nb = 128: j and j + 128) and on other chains
    X = _blobs(20000, 64, 64, seed=75)
    base = X[np.random.default_rng(69).choice(len(X), nb, replace=False)]
    C0 = np.concatenate([base, np.nextafter(base, np.inf)])
    labels = _fit(X, C0, mode)._runner.engine.labels()
    np.testing.assert_array_equal(labels, orc.assign(X, C0)[0])


@pytest.mark.parametrize("mode", MODES)
def test_points_on_and_near_bisectors(mode):
    # close centroid pairs (separation 0.05 .. 5) and points at signed
    # distances 1e-7 .. 1 from their bisector planes, plus tangential noise:
    # the screen's gap is 2 |c_i - c_j| t for a point at distance t
    rng = np.random.default_rng(17)
    d, k = 64, 256
    C0 = rng.uniform(-10, 10, (k, d))
    pairs = rng.permutation(k)[:128].reshape(64, 2)
    for a, b in pairs:
        u = rng.standard_normal(d)
        C0[b] = C0[a] + u / np.linalg.norm(u) * 10 ** rng.uniform(-1.3, 0.7)
    C0 = C0.astype(np.float32).astype(np.float64)
    rows = []
    for a, b in pairs:
        m = 0.5 * (C0[a] + C0[b])
        e = (C0[b] - C0[a]) / np.linalg.norm(C0[b] - C0[a])
        t = np.concatenate([[0.0], 10 ** rng.uniform(-7, 0, 150)]) * rng.choice([-1, 1], 151)
        tang = rng.standard_normal((151, d)) * rng.uniform(0, 3, (151, 1))
        tang -= np.outer(tang @ e, e)
        rows.append(m + tang + np.outer(t, e))
    X = np.concatenate(rows).astype(np.float32).astype(np.float64)
    labels = _fit(X, C0, mode)._runner.engine.labels()
    np.testing.assert_array_equal(labels, orc.assign(X, C0)[0])


@pytest.mark.parametrize("mode", MODES)
def test_far_from_origin(mode):
    # clusters at |c_f| ~ 1000 with unit spread: ||c|| ||x|| is 1e4 x the
    # squared distances, so most points need exact resolution
    X = _blobs(20000, 64, 128, seed=5, box=1000.0, std=1.0)
    C0 = X[np.random.default_rng(2).choice(len(X), 256, replace=False)]
    _check(X, C0, mode)


@pytest.mark.parametrize("mode", MODES)
def test_features_across_magnitudes(mode):
    # feature scales 1e-9 .. 1e3: after the power-of-two scale the small
    # features are fp16 subnormals or zero in the image and the row
    rng = np.random.default_rng(8)
    scale = 10.0 ** np.linspace(-9, 3, 64)
    X = (_blobs(20000, 64, 64, seed=9) * scale).astype(np.float32).astype(np.float64)
    C0 = X[rng.choice(len(X), 200, replace=False)]
    _check(X, C0, mode)


@pytest.mark.parametrize("mode", MODES)
def test_noise_many_iterations(mode):
    rng = np.random.RandomState(42)
    X = rng.randn(30000, 64).astype(np.float32).astype(np.float64)
    C0 = X[np.random.default_rng(2).choice(len(X), 256, replace=False)]
    _check(X, C0, mode, iters=4)


@pytest.mark.parametrize("mode", MODES)
def test_duplicate_centroids_lowest_index(mode):
    X = _blobs(8000, 64, 40, seed=9)
    C0 = X[np.random.default_rng(0).choice(len(X), 256, replace=False)]
    C0[10] = C0[3]
    C0[200] = C0[3]
    labels = _fit(X, C0, mode)._runner.engine.labels()
    np.testing.assert_array_equal(labels, orc.assign(X, C0)[0])
    assert not np.any(labels == 10) and not np.any(labels == 200)


@diag_only
def test_auto_policy_switches_to_fast_screen_and_stays_exact():
    # well separated blobs, one seed per blob: the fp16x3 batch queues almost
    # nothing, so the runtime moves the next batch to the fast screen (policy
    # in km_runtime.hip note_queue); tolerance 0 never converges (strict <,
    # kmeans_spark.py:310), so 40 iterations span several batches (4, 8, 16,
    # 12); the constructor rejects tolerance <= 0 like the reference
    # (kmeans_spark.py:55), so it is set after construction
    ka = _km()
    rng = np.random.default_rng(4)
    centers = rng.uniform(-100, 100, (256, 64))
    lab = rng.integers(0, 256, 40000)
    X = (centers[lab] + 0.5 * rng.standard_normal((40000, 64))).astype(np.float32).astype(np.float64)
    C0 = np.stack([X[np.nonzero(lab == j)[0][0]] for j in range(256)])

    class Pinned(ka.KMeans):
        def _initialize_centroids(self, run):
            return C0.copy()

    km = Pinned(k=256, max_iter=40, tolerance=1e-4, compute_sse=True)
    km.tolerance = 0.0
    km.verbose = False
    km.fit(X)
    assert km._runner.engine.screen() == 2
    # the oracle validates tolerance > 0 like the reference: at 1e-300 it stops
    # at the exact fixed point (shift 0), where the product keeps iterating
    # on unchanged centroids
    ref = orc.lloyd_fit(X, 256, 40, 1e-300, 0, True, 1, init_centroids=C0)
    m = len(ref["sse_history"])
    assert len(km.sse_history) == 40 and m <= 40
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history[:m], ref["sse_history"], rtol=1e-9)
    np.testing.assert_allclose(km.sse_history[m:], [ref["sse_history"][-1]] * (40 - m), rtol=1e-9)
    np.testing.assert_array_equal(km.predict(X).to_numpy(), orc.assign(X, ref["centroids"])[0])


@diag_only
@pytest.mark.parametrize("mode", [2, 3])
@pytest.mark.parametrize("n,d,k", [(20000, 32, 128), (9000, 48, 200)])
def test_fast_modes_fall_back_outside_the_fast_shape(mode, n, d, k):
    # the fast kernel exists for dp = 64, kp = 256 only; elsewhere a forced
    # fast mode runs the fp16x3 fused kernel (km_set_screen): same results
    X = _blobs(n, d, k // 2, seed=d + k)
    C0 = X[np.random.default_rng(4).choice(n, k, replace=False)]
    _check(X, C0, mode)


def test_product_library_rejects_fast_screens():
    if DIAG_LIB:
        pytest.skip("product library only")
    from kmeans_amd import _lib
    from kmeans_amd.engine import make_engine
    from kmeans_amd.comm import Communicator
    eng = make_engine(Communicator())
    with pytest.raises(_lib.KmError, match="diagnostic build only"):
        eng.set_screen(2)
