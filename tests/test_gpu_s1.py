"""The one-MFMA screen with in-kernel re-scoring and delta statistics
(k_s1, km_set_screen mode 4 = KM_SCREEN_S1; csrc/km_screen1.hip).

Reference: kmeans_spark.py:147-159 (np.argmin of np.linalg.norm(C - x,
axis=1), first minimum) and :169-206 (per-cluster sums, mean update).

Bars: labels bit-identical to the oracle's float64 argmin (its NumPy order
and tie-break) -- the screen only proposes candidates, every label it
decides carries a rigorous certificate, the rest go to the float64
resolvers; centroids at 1e-9 relative against the oracle after several
iterations, whose statistics after the first one are carried as deltas (the
rows that changed clusters) on top of the first iteration's full sums.

Predict runs k_s1 in labels-only mode (every geometry with an instance);
fit runs it from the second iteration on (the first one, after new
centroids, runs the fp16x3 screen with full statistics).  compute_sse keeps
the full-statistics screen, so these fits run with it off.
"""
import numpy as np
import pytest

from oracle import kmeans_oracle as orc

pytestmark = pytest.mark.gpu

S1 = 4  # KM_SCREEN_S1 (include/kmeans_amd.h)
SEED = 1234  # empty-cluster repair seed (the reference reads int(time.time()), kmeans_spark.py:196)


def _km():
    import kmeans_amd
    return kmeans_amd


def _engine(mode=-1):
    from kmeans_amd.comm import Communicator
    from kmeans_amd.engine import make_engine
    eng = make_engine(Communicator())
    eng.set_screen(mode)
    return eng


def _predict(X, C, mode=-1):
    eng = _engine(mode)
    eng.load_host(X.astype(np.float32))
    eng.set_centroids(C)
    return eng.predict(), eng


def _fit(X, C0, iters, mode=-1, compute_sse=False):
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

        def _empty_seed(self):
            return SEED

    km = Forced(k=len(C0), max_iter=iters, tolerance=1e-12, compute_sse=compute_sse)
    km.verbose = False
    km.fit(X)
    return km


def _blobs(n, d, centers, seed, box=10.0, std=1.0):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-box, box, (centers, d))
    lab = rng.integers(0, centers, n)
    return (C[lab] + std * rng.standard_normal((n, d))).astype(np.float32).astype(np.float64)


def _check_fit(X, C0, iters):
    km = _fit(X, C0, iters)
    eng = km._runner.engine
    assert eng.screen() == S1, "k_s1 not selected for this geometry"
    ref = orc.lloyd_fit(X, len(C0), iters, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: SEED)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    # labels of the last pass (the centroids it read: those after iters - 1)
    C_prev = orc.lloyd_fit(X, len(C0), iters - 1, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: SEED)["centroids"]
    np.testing.assert_array_equal(eng.labels(), orc.assign(X, C_prev)[0])
    # the sums behind the last update: counts equal the label histogram
    np.testing.assert_array_equal(km._runner.last["counts"], np.bincount(eng.labels(), minlength=len(C0)))
    return km


# -- predict (labels only) on the screen's hard cases --------------------------------

def test_c3_class_selects_s1():
    X = _blobs(4000, 64, 64, seed=1)
    C0 = X[:256].copy()
    km = _fit(X, C0, 2)
    assert km._runner.engine.screen() == S1


@pytest.mark.parametrize("n,d,k,centers", [
    (60000, 64, 256, 256),   # c3 shape: dp 64, kp 256
    (30000, 20, 100, 50),    # dp 32, kp 128 (pads)
    (30000, 32, 250, 300),   # dp 32, kp 256 (8 members per chain, 1 MFMA k-slice)
    (20000, 128, 128, 128),  # dp 128, kp 128
    (20000, 64, 70, 40),     # kp 128, 58 pad slots
    (20000, 32, 384, 200),   # dp 32, kp 384: 12 members per chain (run-time member loop)
    (20000, 32, 512, 300),   # 16 members per chain
    (20000, 32, 1024, 300),  # c4 shape: 32 members, fp32 table in global memory
    (20000, 64, 512, 200),   # dp 64, kp 512: image 64 KiB, table in global memory
])
def test_predict_blobs_vs_oracle(n, d, k, centers):
    X = _blobs(n, d, centers, seed=3 + d)
    C = X[np.random.default_rng(1).choice(n, k, replace=False)]
    labels, _ = _predict(X, C)
    np.testing.assert_array_equal(labels, orc.assign(X, C)[0])


def test_predict_points_on_and_near_bisectors():
    # close centroid pairs (separation 0.05 .. 5) and points at signed
    # distances 1e-7 .. 1 from their bisector planes: exact ties, one-ulp
    # gaps and everything the fp32 re-score must hand to float64
    rng = np.random.default_rng(17)
    d, k = 64, 256
    C = rng.uniform(-10, 10, (k, d))
    pairs = rng.permutation(k)[:128].reshape(64, 2)
    for a, b in pairs:
        u = rng.standard_normal(d)
        C[b] = C[a] + u / np.linalg.norm(u) * 10 ** rng.uniform(-1.3, 0.7)
    C = C.astype(np.float32).astype(np.float64)
    rows = []
    for a, b in pairs:
        m = 0.5 * (C[a] + C[b])
        e = (C[b] - C[a]) / np.linalg.norm(C[b] - C[a])
        t = np.concatenate([[0.0], 10 ** rng.uniform(-7, 0, 150)]) * rng.choice([-1, 1], 151)
        tang = rng.standard_normal((151, d)) * rng.uniform(0, 3, (151, 1))
        tang -= np.outer(tang @ e, e)
        rows.append(m + tang + np.outer(t, e))
    X = np.concatenate(rows).astype(np.float32).astype(np.float64)
    labels, _ = _predict(X, C)
    np.testing.assert_array_equal(labels, orc.assign(X, C)[0])


@pytest.mark.parametrize("nb", [128, 127])
def test_predict_one_ulp_duplicates(nb):
    X = _blobs(20000, 64, 64, seed=75)
    base = X[np.random.default_rng(69).choice(len(X), nb, replace=False)]
    C = np.concatenate([base, np.nextafter(base, np.inf)])
    labels, _ = _predict(X, C)
    np.testing.assert_array_equal(labels, orc.assign(X, C)[0])


def test_predict_duplicate_centroids_lowest_index():
    X = _blobs(8000, 64, 40, seed=9)
    C = X[np.random.default_rng(0).choice(len(X), 256, replace=False)]
    C[10] = C[3]
    C[200] = C[3]
    labels, _ = _predict(X, C)
    np.testing.assert_array_equal(labels, orc.assign(X, C)[0])
    assert not np.any(labels == 10) and not np.any(labels == 200)


def test_predict_far_from_origin():
    # |c_f| ~ 1000, unit spread: the one-MFMA bound (~ 2^-9 ||c|| ||x||) is
    # far wider than the gaps, most rows have more candidates than the
    # kernel re-scores and go to the float64 scan; labels stay exact
    X = _blobs(20000, 64, 128, seed=5, box=1000.0, std=1.0)
    C = X[np.random.default_rng(2).choice(len(X), 256, replace=False)]
    labels, _ = _predict(X, C)
    np.testing.assert_array_equal(labels, orc.assign(X, C)[0])


def test_predict_features_across_magnitudes():
    rng = np.random.default_rng(8)
    scale = 10.0 ** np.linspace(-9, 3, 64)
    X = (_blobs(20000, 64, 64, seed=9) * scale).astype(np.float32).astype(np.float64)
    C = X[rng.choice(len(X), 200, replace=False)]
    labels, _ = _predict(X, C)
    np.testing.assert_array_equal(labels, orc.assign(X, C)[0])


def test_predict_zero_rows_and_zero_centroids():
    # keys of exactly 0 (x = 0, c = 0): packed keys are tiny or signed zeros
    X = _blobs(6000, 64, 32, seed=4)
    X[::7] = 0.0
    C = X[np.random.default_rng(5).choice(len(X), 256, replace=False)]
    C[0] = 0.0
    C[77] = 0.0
    labels, _ = _predict(X, C)
    np.testing.assert_array_equal(labels, orc.assign(X, C)[0])


def test_predict_matches_full_screen_on_many_seeds():
    # the same geometry through k_s1 (auto) and k_fused16 (forced mode 1)
    for seed in range(4):
        X = _blobs(20000, 64, 200, seed=100 + seed)
        C = X[np.random.default_rng(seed).choice(len(X), 256, replace=False)] + 0.3
        a, _ = _predict(X, C, -1)
        b, _ = _predict(X, C, 1)
        np.testing.assert_array_equal(a, b)


# -- fits: delta statistics across iterations ------------------------------------------

def test_fit_c3_shape_delta_iterations():
    X = _blobs(60000, 64, 256, seed=11)
    C0 = X[np.random.default_rng(12).choice(len(X), 256, replace=False)]
    km = _check_fit(X, C0, 8)
    # the certificate settles nearly every row in the kernel (c3 data: about
    # 88% by the screen alone, the rest by the fp32 re-score)
    last = km._runner.last
    assert last["q_full"] + last["q_rerank"] < 0.002 * len(X), last


@pytest.mark.parametrize("iters", [4, 5])
def test_fit_serpentine_delta_iterations_ragged(iters):
    # the c3-class delta fit alternates its sweep (k_s1<2, 8, 1, true> maps the
    # tiles last-first on every other launch where X is <= 8 GiB): even and odd
    # iteration counts end on either direction; a ragged last tile (n % 16 = 7)
    # is first in the descending sweep
    X = _blobs(40_007, 64, 200, seed=21)
    C0 = X[np.random.default_rng(5).choice(len(X), 256, replace=False)]
    _check_fit(X, C0, iters)


def test_fit_noise_delta_iterations():
    # randn: no cluster structure, many rows change clusters every iteration
    rng = np.random.RandomState(42)
    X = rng.randn(30000, 64).astype(np.float32).astype(np.float64)
    C0 = X[np.random.default_rng(2).choice(len(X), 256, replace=False)]
    _check_fit(X, C0, 6)


@pytest.mark.parametrize("n,d,k,centers", [
    (30000, 20, 100, 50),
    (30000, 32, 250, 300),
    (20000, 128, 128, 128),
    (20000, 64, 70, 40),
    (20000, 32, 512, 300),
])
def test_fit_shapes_delta_iterations(n, d, k, centers):
    X = _blobs(n, d, centers, seed=21 + k)
    C0 = X[np.random.default_rng(22).choice(n, k, replace=False)]
    _check_fit(X, C0, 5)


def test_fit_far_from_origin_delta_iterations():
    X = _blobs(20000, 64, 128, seed=5, box=1000.0, std=1.0)
    C0 = X[np.random.default_rng(2).choice(len(X), 256, replace=False)]
    _check_fit(X, C0, 3)


def test_delta_fit_equals_full_statistics_fit():
    # every iteration with full statistics (mode 1: k_fused16) against the
    # default (k_s1 with deltas from the second iteration): identical labels
    # and counts, centroids equal up to float64 summation order
    X = _blobs(40000, 64, 256, seed=31)
    C0 = X[np.random.default_rng(32).choice(len(X), 256, replace=False)]
    a = _fit(X, C0, 6, mode=-1)
    b = _fit(X, C0, 6, mode=1)
    assert a._runner.engine.screen() == S1 and b._runner.engine.screen() == 1
    np.testing.assert_array_equal(a._runner.engine.labels(), b._runner.engine.labels())
    np.testing.assert_array_equal(a._runner.last["counts"], b._runner.last["counts"])
    np.testing.assert_allclose(a.centroids, b.centroids, rtol=1e-12, atol=1e-12)


def test_fit_then_predict_then_fit_again():
    # predict overwrites the labels the deltas refer to: the next fit must
    # start from full statistics again (delta_ready reset), and stay exact
    X = _blobs(20000, 64, 256, seed=41)
    C0 = X[np.random.default_rng(42).choice(len(X), 256, replace=False)]
    km = _fit(X, C0, 3)
    run = km._runner
    km.predict(X)
    km.max_iter = 3
    run.engine.set_centroids(np.asarray(km.centroids, dtype=np.float64))
    run.run(km, None, 3)
    C3 = orc.lloyd_fit(X, 256, 3, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: SEED)["centroids"]
    ref = orc.lloyd_fit(X, 256, 3, 1e-12, 0, False, 1, init_centroids=C3, empty_seed=lambda: SEED)
    np.testing.assert_allclose(run.engine.get_centroids(0), ref["centroids"], rtol=1e-9, atol=1e-9)


def test_long_delta_fit_no_drift_vs_full_statistics():
    # the bench's steady state is a long run of delta iterations (the reference
    # default is max_iter = 100, kmeans_spark.py:37): the full sums under the
    # deltas are carried across every iteration of the fit, never re-based.
    # 100 iterations on unstructured data at the c3 geometry (rows keep moving
    # between clusters, tolerance 1e-300 never converges): identical labels and
    # counts to the fit that recomputes full statistics every iteration
    # (mode 1), centroids within float64 summation order of it, and the final
    # centroids equal the float64 means of the rows under the final labels
    # (np.add.at in the oracle's dtype), to 1e-9
    rng = np.random.RandomState(7)
    X = rng.randn(200_000, 64).astype(np.float32).astype(np.float64)
    C0 = X[np.random.default_rng(8).choice(len(X), 256, replace=False)]
    iters = 100
    ka = _km()

    def fit(mode):
        from kmeans_amd.engine import make_engine

        def factory(comm):
            eng = make_engine(comm)
            eng.set_screen(mode)
            return eng

        class Forced(ka.KMeans):
            _engine_factory = staticmethod(factory)

            def _initialize_centroids(self, run):
                return C0.copy()

            def _empty_seed(self):
                return SEED

        km = Forced(k=256, max_iter=iters, tolerance=1e-300, compute_sse=False)
        km.verbose = False
        km.fit(X)
        return km

    a, b = fit(-1), fit(1)
    ea, eb = a._runner.engine, b._runner.engine
    assert a._runner.iterations_ran == iters == b._runner.iterations_ran
    assert ea.screen() == S1 and ea.info()["delta_stats"] == 1
    assert eb.info()["delta_stats"] == 0
    la = ea.labels()
    np.testing.assert_array_equal(la, eb.labels())
    np.testing.assert_array_equal(a._runner.last["counts"], b._runner.last["counts"])
    np.testing.assert_allclose(a.centroids, b.centroids, rtol=1e-12, atol=1e-12)
    counts = np.bincount(la, minlength=256)
    np.testing.assert_array_equal(a._runner.last["counts"], counts)
    sums = np.zeros((256, 64))
    np.add.at(sums, la, X)
    nz = counts > 0
    np.testing.assert_allclose(a.centroids[nz], sums[nz] / counts[nz, None], rtol=1e-9, atol=1e-9)
    # the last assignment against the oracle (the centroids it read are the
    # ones before the last update: run one more oracle-free check on labels)
    C_prev = ea.get_centroids(0)      # after the last update = the next pass's input
    np.testing.assert_array_equal(ea.predict(), orc.assign(X, C_prev)[0])


@pytest.mark.parametrize("n,d,k,centers", [
    (20000, 18, 1000, 300),   # dp 32, kp 1024 (unfused): k (d+1) 8 + the wave prefix fit LDS -> LDS aggregation
    (20000, 19, 1000, 300),   # dp 32, kp 1024: 160,000 B of table + the prefix do not fit -> two cluster ranges
    (20000, 60, 480, 200),    # dp 64, kp 512 (unfused): cluster ranges
])
def test_unfused_geometries_delta_statistics(n, d, k, centers):
    # every k_s1 geometry takes delta statistics (round 6): k_s1_delta
    # aggregates the changed rows in an LDS [k][d+1] table where it fits
    # beside the largest grid's wave prefix (geometry and device only, never
    # the rank's rows), else over cluster ranges whose tables fit; the
    # resolvers write their rows' moves into the same change list
    X = _blobs(n, d, centers, seed=21 + k + d)
    C0 = X[np.random.default_rng(22).choice(n, k, replace=False)]
    km = _check_fit(X, C0, 5)
    info = km._runner.engine.info()
    assert info["fused_stats"] == 0
    assert info["delta_stats"] == 1


def test_assign_stats_twice_before_update():
    # a caller that runs km_assign_stats twice before km_update:
    # the first call's deltas were never folded, so the second computes full
    # sums; the update then matches the oracle's one step, and later delta
    # iterations stay exact
    X = _blobs(30000, 64, 256, seed=91)
    C0 = X[np.random.default_rng(92).choice(len(X), 256, replace=False)]
    km = _fit(X, C0, 3)
    run, eng = km._runner, km._runner.engine
    C3 = eng.get_centroids(0)
    eng.assign_stats()
    assert eng.info()["delta_stats"] == 1
    eng.assign_stats()
    assert eng.info()["delta_stats"] == 0
    st, counts = eng.update()
    ref = orc.lloyd_fit(X, 256, 1, 1e-12, 0, False, 1, init_centroids=C3, empty_seed=lambda: SEED)
    np.testing.assert_allclose(eng.get_centroids(1), ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_array_equal(counts, np.bincount(orc.assign(X, C3)[0], minlength=256))
    eng.commit()
    km.max_iter = 6
    run.run(km, None, 6, first=4)
    assert eng.info()["delta_stats"] == 1
    ref2 = orc.lloyd_fit(X, 256, 2, 1e-12, 0, False, 1, init_centroids=ref["centroids"], empty_seed=lambda: SEED)
    np.testing.assert_allclose(eng.get_centroids(0), ref2["centroids"], rtol=1e-9, atol=1e-9)


def test_predict_between_assign_and_update_keeps_the_deltas():
    # predict after a delta km_assign_stats and before its update: the update
    # still folds that assignment's deltas (same centroids, same labels)
    X = _blobs(30000, 64, 256, seed=93)
    C0 = X[np.random.default_rng(94).choice(len(X), 256, replace=False)]
    km = _fit(X, C0, 3)
    eng = km._runner.engine
    C3 = eng.get_centroids(0)
    eng.assign_stats()
    assert eng.info()["delta_stats"] == 1
    np.testing.assert_array_equal(eng.predict(), orc.assign(X, C3)[0])
    st, counts = eng.update()
    ref = orc.lloyd_fit(X, 256, 1, 1e-12, 0, False, 1, init_centroids=C3, empty_seed=lambda: SEED)
    np.testing.assert_allclose(eng.get_centroids(1), ref["centroids"], rtol=1e-9, atol=1e-9)


def test_compute_sse_with_delta_statistics():
    # compute_sse no longer forces full statistics (round 6): from the second
    # iteration k_s1 adds every decided row's float64 residual to the fp32
    # image c' of its centroid, the resolvers the queued rows', and the update
    # adds the exact per-cluster correction -2 dl (S - n c') + n dl^2
    # (dl = c - c'), so the SSE is the reference's sum of min(norm)**2
    # (kmeans_spark.py:224-237) with one read of the rows per iteration
    X = _blobs(20000, 64, 256, seed=51)
    C0 = X[np.random.default_rng(52).choice(len(X), 256, replace=False)]
    km = _fit(X, C0, 4, compute_sse=True)
    eng = km._runner.engine
    assert eng.screen() == S1 and eng.info()["delta_stats"] == 1
    ref = orc.lloyd_fit(X, 256, 4, 1e-12, 0, True, 1, init_centroids=C0, empty_seed=lambda: SEED)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)


@pytest.mark.parametrize("n,d,k,centers", [
    (12000, 64, 256, 64),     # c3 geometry: LDS delta table, fp32 table in LDS
    (12000, 32, 1024, 256),   # c4 geometry: deltas over two cluster ranges, fp32 table in global memory
])
def test_tight_clusters_sse_delta_iterations(n, d, k, centers):
    # std 1e-3 in a +-1000 box (sum ||x||^2 ~ 1e12 x the SSE): the residuals to
    # c' and the per-cluster correction must hold 1e-9 where any closed form
    # through ||x||^2 cancels; the screen's bound is wide here, so most rows
    # reach the float64 resolvers, which add their residuals the same way
    rng = np.random.default_rng(d + k)
    C = rng.uniform(-1000, 1000, (centers, d))
    blob = rng.integers(0, centers, n)
    X = (C[blob] + 1e-3 * rng.standard_normal((n, d))).astype(np.float32).astype(np.float64)
    first = [int(np.nonzero(blob == b)[0][0]) for b in range(centers) if np.any(blob == b)]
    rest = np.setdiff1d(np.arange(n), first)
    C0 = X[np.concatenate([first, rng.choice(rest, k - len(first), replace=False)]).astype(np.int64)]
    km = _fit(X, C0, 4, compute_sse=True)
    eng = km._runner.engine
    assert eng.screen() == S1 and eng.info()["delta_stats"] == 1
    ref = orc.lloyd_fit(X, k, 4, 1e-12, 0, True, 1, init_centroids=C0, empty_seed=lambda: SEED)
    assert ref["sse_history"][-1] < 1e-4 * np.sum(X * X)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)


# -- the unfused geometries (c4 class): k_s1 labels, then the statistics pass ------------

@pytest.mark.parametrize("compute_sse", [True, False])
def test_fit_c4_shape_labels_then_statistics_pass(compute_sse):
    # k = 1024, d = 32 (c4's geometry; BASELINE configs[3] has compute_sse on):
    # no fused statistics table fits, so the first iteration is k_s1's labels
    # and the statistics pass (with the SSE residuals); from the second on,
    # delta statistics folded over cluster ranges (the [k][d+1] table does
    # not fit LDS) and the residuals in k_s1: one read of X per iteration
    X = _blobs(30000, 32, 1024, seed=61)
    C0 = X[np.random.default_rng(62).choice(len(X), 1024, replace=False)]
    km = _fit(X, C0, 4, compute_sse=compute_sse)
    eng = km._runner.engine
    assert eng.screen() == S1 and eng.info()["delta_stats"] == 1
    ref = orc.lloyd_fit(X, 1024, 4, 1e-12, 0, compute_sse, 1, init_centroids=C0, empty_seed=lambda: SEED)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    if compute_sse:
        np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
    C_prev = orc.lloyd_fit(X, 1024, 3, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: SEED)["centroids"]
    np.testing.assert_array_equal(eng.labels(), orc.assign(X, C_prev)[0])


def test_c4_shape_forced_fp16x3_screen_still_available():
    # km_set_screen(1) keeps the fp16x3 unfused screen on this geometry
    X = _blobs(20000, 32, 1024, seed=63)
    C = X[np.random.default_rng(64).choice(len(X), 1024, replace=False)]
    a, eng = _predict(X, C, 1)
    assert eng.screen() == 1
    np.testing.assert_array_equal(a, orc.assign(X, C)[0])


# -- KM_SCREEN_ONE: one fp16 MFMA per product in the unfused k_assign_mfma16 -------------

ONE = 5  # KM_SCREEN_ONE (include/kmeans_amd.h)


@pytest.mark.parametrize("n,d,k,centers", [
    (8000, 128, 4096, 512),   # c5 geometry: chunked images, top-2 chains (dp 128)
    (12000, 64, 1536, 300),   # dp 64, chunked, top-3 chains
    (12000, 96, 640, 200),    # dp 96 (not a multiple of 32): the fp16x3 32x32x16 screen stays
])
def test_one_mfma_unfused_screen_predict_vs_oracle(n, d, k, centers):
    X = _blobs(n, d, centers, seed=70 + d)
    C = X[np.random.default_rng(71).choice(n, k, replace=False)]
    a, eng = _predict(X, C)
    np.testing.assert_array_equal(a, orc.assign(X, C)[0])
    assert eng.screen() == (ONE if d % 32 == 0 else 1)
    b, _ = _predict(X, C, 1)
    np.testing.assert_array_equal(a, b)


def test_one_mfma_unfused_screen_fit_c5_shape():
    # the c5 geometry (d 128, k 4096) through fit: labels, then the sorted
    # statistics pass; centroids and SSE against the oracle
    X = _blobs(12000, 128, 1024, seed=81)
    C0 = X[np.random.default_rng(82).choice(len(X), 4096, replace=False)]
    km = _fit(X, C0, 3, compute_sse=True)
    assert km._runner.engine.screen() == ONE
    ref = orc.lloyd_fit(X, 4096, 3, 1e-12, 0, True, 1, init_centroids=C0, empty_seed=lambda: SEED)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)


@pytest.mark.parametrize("n,d,k,centers,iters", [
    (12000, 128, 4096, 1024, 4),  # c5 geometry: chunked images, one-MFMA screen, deltas over 29 cluster ranges
    (12000, 64, 1536, 300, 5),    # dp 64, kp 1536 (no k_s1 instance): the same screen and deltas
])
def test_one_mfma_unfused_screen_delta_statistics(n, d, k, centers, iters):
    # the unfused k_assign_mfma16 geometries take delta statistics too (round
    # 6, compute_sse off): from the second iteration the screen lists the rows
    # whose label changed, the resolvers move their changed rows, and
    # k_s1_delta folds the list -- no statistics pass over X
    X = _blobs(n, d, centers, seed=83 + d)
    C0 = X[np.random.default_rng(84).choice(len(X), k, replace=False)]
    km = _fit(X, C0, iters)
    eng = km._runner.engine
    assert eng.screen() == ONE and eng.info()["delta_stats"] == 1
    ref = orc.lloyd_fit(X, k, iters, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: SEED)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    C_prev = orc.lloyd_fit(X, k, iters - 1, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: SEED)["centroids"]
    np.testing.assert_array_equal(eng.labels(), orc.assign(X, C_prev)[0])
    np.testing.assert_array_equal(km._runner.last["counts"], np.bincount(eng.labels(), minlength=k))


def test_one_mfma_unfused_poor_seeds_delta_statistics():
    # c5's poor seeds (3 data rows + far points: mass empties repaired on the
    # device at iteration 1), then delta iterations over the repaired
    # centroids, against the oracle's whole loop (pinned repair seed)
    n, d, k = 12000, 128, 1024
    X = _blobs(n, d, 64, seed=57)
    far = np.full((k - 3, d), 100.0) + np.arange(k - 3)[:, None]
    C0 = np.vstack([X[[0, 1, 2]], far])
    km = _fit(X, C0, 4)
    eng = km._runner.engine
    assert eng.info()["delta_stats"] == 1 and km._runner.device_repairs >= 1
    ref = orc.lloyd_fit(X, k, 4, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: SEED)
    assert ref["records"][0]["empty"]
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)


# -- the full scans' fp32 prefilter (k_fullscan<..., PF>) ---------------------------------

@pytest.mark.parametrize("d,k,group", [
    (128, 4096, 20),   # c5 geometry: <= 64 kept, float64 on the kept ones
    (128, 4096, 80),   # more than 64 kept: the float64 chunk pass
    (64, 256, 24),     # c3 geometry (k_s1's full scans)
    (32, 1024, 40),    # c4 geometry
    (96, 640, 30),     # dp 96: the fp16x3 screen's full scans
])
def test_full_scan_prefilter_equidistant_groups(d, k, group):
    # rows with a group of centroids at the same distance up to float64
    # rounding: no screen separates them, the full scan's fp32 prefilter keeps
    # the whole group (its bounds overlap), and the float64 NumPy-order norms
    # pick the reference's argmin -- including the lowest-index tie-break
    rng = np.random.default_rng(d + k + group)
    nrow = 3000
    X = rng.uniform(-5, 5, (nrow, d)).astype(np.float32).astype(np.float64)
    C = rng.uniform(-5, 5, (k, d))
    ng = min(64, k // group)
    for i in range(ng):
        u = rng.standard_normal((group, d))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        C[i * group:(i + 1) * group] = X[i] + 0.5 * u
    C[ng * group] = C[0]  # an exact duplicate: the lower index wins
    a, eng = _predict(X, C)
    np.testing.assert_array_equal(a, orc.assign(X, C)[0])


@pytest.mark.parametrize("d,k", [(128, 4096), (64, 1536), (64, 256)])
def test_rerank_prefilter_relative_gaps(d, k):
    # rows whose two nearest centroids differ in distance by a relative gap
    # around the fp32 prefilter's margin (8u = 4.8e-7 and its bounds' e):
    # below it both stay for float64, above it one is kept and decides alone;
    # labels must be the oracle's on both sides (and for exact ties)
    rng = np.random.default_rng(d + k + 7)
    nrow = 4000
    X = rng.uniform(-5, 5, (nrow, d)).astype(np.float32).astype(np.float64)
    C = rng.uniform(-5, 5, (k, d)) * 3.0
    gaps = [0.0, 1e-9, 1e-7, 3e-7, 1e-6, 3e-6, 1e-5, 1e-4]
    npairs = min(nrow, k // 2)
    for i in range(npairs):
        u = rng.standard_normal((2, d))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        r = 0.7
        gap = gaps[i % len(gaps)]
        C[2 * i] = X[i] + r * u[0]
        C[2 * i + 1] = X[i] + r * (1.0 + gap) * u[1]
        if i % 2:
            C[[2 * i, 2 * i + 1]] = C[[2 * i + 1, 2 * i]]  # the nearer one at the higher index half the time
    a, eng = _predict(X, C)
    np.testing.assert_array_equal(a, orc.assign(X, C)[0])
