"""GPU parity: the HIP path (through the C-ABI) against the reference's golden
vectors and the CPU oracle.

Bars (BASELINE.json north_star): labels bit-exact except where the reference's
top-2 distances differ by < 1e-6 relative; centroids within 1e-5 relative;
SSE within 1e-6 relative.  The exact-resolve design aims much tighter (the
assertions below use 1e-9 where the float64 re-rank makes that the expected
agreement; the north-star bars are asserted too).
"""
import contextlib
import io
import re

import numpy as np
import pytest

from conftest import F32_CASES, GOLDEN_CASES, check_float32_run
from oracle import kmeans_oracle as orc

pytestmark = pytest.mark.gpu

RTOL_C = 1e-5     # north-star centroid bar
RTOL_SSE = 1e-6   # north-star SSE bar
BAND = 1e-6       # north-star label band


def _km():
    import kmeans_amd
    return kmeans_amd


def _fit_product(g, inject=True, slices=None, dtype=None):
    ka = _km()
    init = g["init"]

    class Pinned(ka.KMeans):
        def _initialize_centroids(self, run):
            if inject:
                return init.copy()
            return super()._initialize_centroids(run)

        def _empty_seed(self):
            return int(g["time_seed"])

    sc = ka.LocalContext()
    rdd = sc.parallelize(g["X"] if dtype is None else g["X"].astype(dtype), slices or int(g["slices"]))
    km = Pinned(k=int(g["k"]), max_iter=int(g["max_iter"]), tolerance=float(g["tol"]), seed=int(g["seed"]),
                compute_sse=bool(g["sse"]))
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        km.fit(rdd, sc)
    labels = np.array(km.predict(rdd, sc).collect())
    return km, buf.getvalue(), labels


def _lines(s):
    return [ln for ln in s.splitlines() if ln.strip()]


_NUM = re.compile(r"[-+]?\d+\.\d+")


def assert_logs_match(ours, ref):
    a, b = _lines(ours), _lines(ref)
    assert len(a) == len(b), f"log length {len(a)} != {len(b)}\nours:\n{ours}\nref:\n{ref}"
    for x, y in zip(a, b):
        # identical text except the last printed digit of floats may differ
        assert _NUM.sub("#", x) == _NUM.sub("#", y), (x, y)
        for u, v in zip(_NUM.findall(x), _NUM.findall(y)):
            assert abs(float(u) - float(v)) <= 2 * 10 ** -len(v.split(".")[1]) + 1e-9 * abs(float(v)), (x, y)


@pytest.mark.parametrize("name", F32_CASES)
def test_float32_rows_meet_the_bars_against_the_reference_float32_run(golden, name):
    # the reference on float32 rows computes in float32; the product in
    # float64 on the same rows (centroids returned as float32)
    g = golden(name)
    km, out, labels = _fit_product(g, dtype=np.float32)
    check_float32_run(g, km.centroids, km.sse_history, labels, out)
    # and the product's own contract: the float64 run on those rows
    ref = orc.lloyd_fit(g["X"], int(g["k"]), int(g["max_iter"]), float(g["tol"]), int(g["seed"]), True,
                        int(g["slices"]), init_centroids=g["init"], empty_seed=lambda: int(g["time_seed"]))
    np.testing.assert_allclose(km.centroids, ref["centroids"].astype(np.float32), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_fit_matches_reference_golden(golden, name):
    g = golden(name)
    km, out, labels = _fit_product(g)
    ref_c = g["centroids"]
    np.testing.assert_allclose(km.centroids, ref_c, rtol=RTOL_C, atol=1e-9)
    np.testing.assert_allclose(km.centroids, ref_c, rtol=1e-9, atol=1e-9)
    assert len(km.sse_history) == len(g["sse_history"])
    np.testing.assert_allclose(km.sse_history, g["sse_history"], rtol=RTOL_SSE)
    np.testing.assert_allclose(km.sse_history, g["sse_history"], rtol=1e-9)
    assert_logs_match(out, g["stdout"])
    assert km.iterations_run == int(g["iterations_run"]) == 0
    np.testing.assert_array_equal(labels, g["labels"])
    assert all(type(v) is int for v in km.predict(g["X"]).collect()[:10])


@pytest.mark.parametrize("name", ["test_a", "test_c", "test_d", "c2_small"])
def test_takesample_init_policy_matches_reference(golden, name):
    g = golden(name)
    km, out, labels = _fit_product(g, inject=False)
    np.testing.assert_allclose(km.centroids, g["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_array_equal(labels, g["labels"])


def _blobs(n, d, centers, seed, box=10.0, std=1.0, with_labels=False):
    rng = np.random.default_rng(seed)
    C = rng.uniform(-box, box, (centers, d))
    lab = rng.integers(0, centers, n)
    X = (C[lab] + std * rng.standard_normal((n, d))).astype(np.float32).astype(np.float64)
    return (X, lab) if with_labels else X


def _one_step(X, C0, compute_sse=True, iters=1, screen=-1):
    ka = _km()
    from kmeans_amd.engine import make_engine

    def factory(comm):
        eng = make_engine(comm)
        eng.set_screen(screen)
        return eng

    class Pinned(ka.KMeans):
        _engine_factory = staticmethod(factory)

        def _initialize_centroids(self, run):
            return C0.copy()

    km = Pinned(k=len(C0), max_iter=iters, tolerance=1e-12, compute_sse=compute_sse)
    km.verbose = False
    km.fit(X)
    return km


def _check_labels(X, C, labels):
    lab_ref, _, gap = orc.assign(X, C)
    bad = np.nonzero(labels != lab_ref)[0]
    assert np.all(gap[bad] < BAND), f"{len(bad)} label mismatches outside the 1e-6 band"
    return len(bad)


@pytest.mark.parametrize("n,d,k,centers", [
    (50000, 64, 256, 256),     # c3 shape (MFMA path)
    (20000, 32, 1024, 1024),   # c4 shape (MFMA path, 8-wave workgroups)
    (30000, 16, 8, 8),         # c2 shape (small path)
    (6000, 128, 4096, 512),    # c5 shape (chunked centroids)
    (20000, 3, 5, 3),          # odd d
    (12345, 17, 40, 10),       # d=17 -> 32 padded, k not a multiple of 32
    (9999, 100, 70, 20),       # d=100 -> 128 padded
    (4000, 200, 33, 33),       # d=200 -> 256 padded
    (40, 64, 36, 8),           # two 32-point tiles, the second partial (fused kernel tail)
    (1000, 40, 70, 10),        # d=40 -> 48 padded (fused <3,4>, generic row norms)
    (5000, 64, 300, 60),       # k=300 -> kp=320: unfused MFMA path + LDS-range statistics
    (6000, 128, 1200, 100),    # statistics tiled over 2 cluster ranges x 8 feature ranges
    (4000, 40, 300, 30),       # dp 48 unfused: k_stats lane groups of 12 (4 lanes idle)
    (4000, 90, 200, 30),       # dp 96 unfused: lane groups of 24
    (3000, 180, 150, 30),      # dp 192 unfused: lane groups of 48
    (6000, 300, 70, 20),       # d=300 -> 304: feature-piece screen (k_assign_wide), one centroid chunk, last piece 48 wide
    (3000, 784, 200, 40),      # d=784: 13 feature pieces (last one 16 wide), statistics over 196-wide ranges
    (2000, 300, 700, 50),      # wide rows, 3 centroid chunks (the last 192 wide), 3 cluster ranges
])
def test_one_step_vs_oracle(n, d, k, centers):
    X = _blobs(n, d, centers, seed=n + d + k)
    rng = np.random.default_rng(1)
    C0 = X[rng.choice(n, k, replace=False)]
    km = _one_step(X, C0)
    ref = orc.lloyd_fit(X, k, 1, 1e-12, 0, True, 1, init_centroids=C0)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
    labels = km.predict(X).to_numpy()
    assert _check_labels(X, ref["centroids"], labels) == 0


@pytest.mark.parametrize("n,d,k,slices", [(30000, 16, 12, 4), (20000, 100, 40, 3)])
def test_raw_float64_input_is_the_reference_on_its_fp32_rounding(n, d, k, slices):
    # raw float64 make_blobs-style rows (not fp32-representable).  The compute
    # contract (KMeans docstring): rows are rounded to float32
    # once at load and every row the fit uses -- assignment, sums, the
    # takeSample initial centroids -- is the rounded row.  So the result IS the
    # reference's on X.astype(float32) (bit-exact labels, 1e-9 centroids/SSE),
    # and within float32 rounding of the reference's on the raw rows.
    ka = _km()
    rng = np.random.default_rng(n + d)
    centers = rng.uniform(-10, 10, (k, d))
    X = centers[rng.integers(0, k, n)] + rng.standard_normal((n, d))
    assert not np.array_equal(X, X.astype(np.float32).astype(np.float64))
    class Seeded(ka.KMeans):
        def _empty_seed(self):          # int(time.time()) at L196, pinned for the comparison
            return 1234

    km = Seeded(k=k, max_iter=8, tolerance=1e-4, seed=11, compute_sse=True)
    km.verbose = False
    rdd = ka.LocalContext().parallelize(X, slices)
    km.fit(rdd)
    labels = np.asarray(km.predict(rdd).collect())
    X32 = X.astype(np.float32).astype(np.float64)
    ref32 = orc.lloyd_fit(X32, k, 8, 1e-4, 11, True, slices, empty_seed=lambda: 1234)
    np.testing.assert_allclose(km.centroids, ref32["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref32["sse_history"], rtol=1e-9)
    np.testing.assert_array_equal(labels, orc.assign(X32, ref32["centroids"])[0])
    # against the raw-float64 reference: same run, float32-rounding close
    ref64 = orc.lloyd_fit(X, k, 8, 1e-4, 11, True, slices, empty_seed=lambda: 1234)
    assert len(ref64["sse_history"]) == len(km.sse_history)
    np.testing.assert_allclose(km.centroids, ref64["centroids"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(km.sse_history, ref64["sse_history"], rtol=1e-6)
    lab64, _, gap = orc.assign(X, ref64["centroids"])
    bad = np.nonzero(labels != lab64)[0]
    assert np.all(gap[bad] < BAND), f"{len(bad)} label mismatches outside the 1e-6 band"


def test_load_rows_multi_chunk_staging():
    # km_load_rows streams through two 64 MiB pinned halves (262,144 rows of
    # d = 64 each): rows at and around the chunk boundaries come back exactly,
    # column sums match (float32 rows, float64 sums)
    from kmeans_amd.engine import HipEngine
    rng = np.random.default_rng(9)
    n, d = 700_001, 64
    X = rng.standard_normal((n, d)).astype(np.float32)
    eng = HipEngine(0)
    try:
        eng.load_host(X)
        per = (16 << 20) // d
        idx = np.array([0, per - 1, per, per + 1, 2 * per - 1, 2 * per, n - 1], dtype=np.int64)
        np.testing.assert_array_equal(eng.gather_rows(idx), X[idx].astype(np.float64))
        np.testing.assert_allclose(eng.sum_x(), X.astype(np.float64).sum(axis=0), rtol=1e-9, atol=1e-6)
    finally:
        eng.close()


def test_randn_many_iterations_vs_oracle():
    # random noise (test_b style): many near-ties, stresses the exact resolve
    rng = np.random.RandomState(42)
    X = rng.randn(40000, 64).astype(np.float32).astype(np.float64)
    C0 = X[np.random.default_rng(2).choice(len(X), 256, replace=False)]
    km = _one_step(X, C0, iters=4)
    ref = orc.lloyd_fit(X, 256, 4, 1e-12, 0, True, 1, init_centroids=C0)
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)


def test_duplicate_centroids_tie_break_lowest_index():
    X = _blobs(5000, 64, 40, 9)
    C0 = X[np.random.default_rng(0).choice(5000, 64, replace=False)]
    C0[10] = C0[3]          # exact duplicate: np.argmin picks 3
    C0[50] = C0[3]
    labels = _one_step(X, C0, iters=1)._runner.engine.labels()
    lab_ref = orc.assign(X, C0)[0]
    np.testing.assert_array_equal(labels, lab_ref)
    assert not np.any(labels == 10) and not np.any(labels == 50)


def test_nan_data_raises_like_reference():
    X = _blobs(3000, 8, 4, 1)
    C0 = X[:4].copy()
    X[100, 2] = np.nan
    with pytest.raises(ValueError, match=r"NaN or Inf detected in centroids at iteration 1"):
        _one_step(X, C0)


def test_k_larger_than_n_raises():
    ka = _km()
    with pytest.raises(ValueError, match=r"Not enough data points \(5\) to initialize 6 clusters"):
        ka.KMeans(k=6).fit(np.zeros((5, 2)))


def test_predict_requires_fit():
    ka = _km()
    with pytest.raises(ValueError, match="Model must be fitted before prediction"):
        ka.KMeans(k=2).predict(np.zeros((5, 2)))


@pytest.mark.parametrize("n,d,nb,off", [
    (20000, 64, 128, 128),   # fused kernel, duplicates on the same chain -> full scans
    (20000, 64, 127, 127),   # fused kernel, duplicates on other chains -> pair re-rank
    (20000, 16, 12, 12),     # small path (k <= 32): in-thread re-rank / full scan
    (8000, 100, 150, 150),   # unfused MFMA path (kp = 320)
    (8000, 32, 300, 300),    # unfused, top-2 chains (d <= 32), duplicates on other chains -> re-rank
    (8000, 32, 264, 264),    # unfused, top-2 chains, duplicates on the same chain -> full scans
    (6000, 200, 40, 40),     # d = 200: pairwise split 96 + 104
    (6000, 250, 20, 20),     # d = 250: split 120 + (64 + 66), two levels
    (3000, 300, 40, 40),     # d = 300: wide re-rank (k_rerank2<true>), three levels
    (2000, 784, 24, 24),     # d = 784: 392 + 392 -> ... five levels
])
def test_near_ties_one_ulp_apart_vs_oracle(n, d, nb, off):
    # centroids duplicated and nudged by one float64 ulp: every point is a
    # near-tie the screen cannot separate; the float64 resolvers must return
    # np.argmin over np.linalg.norm bit for bit (kmeans_spark.py:153-156)
    X = _blobs(n, d, 64, 11 + d)
    rng = np.random.default_rng(5 + d)
    base = X[rng.choice(len(X), nb, replace=False)]
    C0 = np.concatenate([base, np.nextafter(base, np.inf)])
    assert len(C0) == nb + off
    labels = _one_step(X, C0, iters=1)._runner.engine.labels()
    lab_ref = orc.assign(X, C0)[0]
    np.testing.assert_array_equal(labels, lab_ref)


@pytest.mark.parametrize("n,d,nb,copies,top3", [
    (8000, 100, 100, 3, True),    # dp 128 (top-3 chains), kp 320: copies on other and on the same chain
    (8000, 64, 81, 4, True),      # four ulp-copies on four chains (kp 384, unfused)
    (8000, 64, 80, 4, False),     # four copies on ONE chain (80 = 0 mod 8): the guard overflows -> full scan
    (6000, 32, 100, 3, False),    # top-2 chains (d <= 32): two copies on one chain overflow -> full scan
    (4000, 128, 601, 3, True),    # k = 1803: chunked centroid images (c5 class)
])
@pytest.mark.parametrize("screen", [1, -1])
def test_candidate_lists_multi_ties_vs_oracle(n, d, nb, copies, top3, screen):
    # three or four centroids one float64 ulp apart: no pair certificate (kind
    # 2).  The MFMA screen lists the chains' kept keys within the bound
    # (kind 4) when no chain's guard key is within it, and k_rerank2 resolves
    # the list in float64 -- labels must be np.argmin over np.linalg.norm bit
    # for bit, and the candidate lists must replace most full scans
    X = _blobs(n, d, 32, 41 + d)
    base = X[np.random.default_rng(d + nb).choice(n, nb, replace=False)]
    cs = [base]
    for _ in range(copies - 1):
        cs.append(np.nextafter(cs[-1], np.inf))
    C0 = np.concatenate(cs)
    km = _one_step(X, C0, iters=1, screen=screen)
    lab_ref = orc.assign(X, C0)[0]
    np.testing.assert_array_equal(km._runner.engine.labels(), lab_ref)
    # (the copies that win no point are empty clusters, replaced by a
    # time-seeded takeSample: only the labels and the SSE are deterministic)
    ref = orc.lloyd_fit(X, len(C0), 1, 1e-12, 0, True, 1, init_centroids=C0)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
    last = km._runner.last
    assert last["q_rerank"] + last["q_full"] > n // 2          # nearly every point is a multi-tie
    if top3 and screen == 1:
        # the fp16x3 screen's narrow bound: the lists hold the copies alone
        # (the default screens on these geometries, k_s1 and the one-MFMA
        # k_assign_mfma16, bound ~2^-11 instead of ~2^-22: their lists also
        # take in neighbouring groups and overflow more often, a cost only)
        assert last["q_full"] < n // 4, last                 # most go to candidate lists, not full scans


@pytest.mark.parametrize("n,d,nb", [(3000, 300, 30), (1500, 784, 16), (1200, 2000, 8)])
def test_wide_rows_triple_ties_full_scan_vs_oracle(n, d, nb):
    # three centroids one float64 ulp apart: no re-rank certificate, so the
    # points go to the wide full scan (k_fullscan<2, true>, C64T from L2);
    # labels must be np.argmin over np.linalg.norm bit for bit
    X = _blobs(n, d, 16, 29 + d)
    base = X[np.random.default_rng(d).choice(n, nb, replace=False)]
    up = np.nextafter(base, np.inf)
    C0 = np.concatenate([base, up, np.nextafter(up, np.inf)])
    km = _one_step(X, C0, iters=1)
    lab_ref = orc.assign(X, C0)[0]
    np.testing.assert_array_equal(km._runner.engine.labels(), lab_ref)
    ref = orc.lloyd_fit(X, len(C0), 1, 1e-12, 0, True, 1, init_centroids=C0)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)


@pytest.mark.parametrize("n,d,k,centers", [
    (20000, 16, 8, 8),          # c2 shape: small path, residuals fused in k_assign_small
    (20000, 64, 256, 256),      # c3 shape: fused kernel, residuals in the same pass + resolvers
    (12000, 32, 1024, 256),     # c4 shape: unfused MFMA path, residuals in k_stats
    (12000, 128, 4096, 512),    # c5 shape: label-sorted statistics, residuals fused in k_segsum
    (5000, 64, 300, 60),        # unfused, LDS-range statistics with residuals
])
def test_tight_clusters_sse_vs_oracle(n, d, k, centers):
    # std 1e-3 in a +-1000 box: sum ||x||^2 is ~1e12 x the SSE.  The reference
    # sums min(norm)**2 per point (kmeans_spark.py:224-237); a closed form
    # through ||x||^2 loses ~1e-5 relative here (north-star bar 1e-6)
    X, blob = _blobs(n, d, centers, seed=7 + d, box=1000.0, std=1e-3, with_labels=True)
    first = [int(np.nonzero(blob == b)[0][0]) for b in range(centers)]
    rest = np.setdiff1d(np.arange(n), first)
    extra = np.random.default_rng(3).choice(rest, k - centers, replace=False) if k > centers else []
    C0 = X[np.concatenate([first, extra]).astype(np.int64)]
    km = _one_step(X, C0)
    ref = orc.lloyd_fit(X, k, 1, 1e-12, 0, True, 1, init_centroids=C0)
    assert ref["sse_history"][0] < 1e-4 * np.sum(X * X)   # the regime that cancels
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
    if not ref["records"][0]["empty"]:
        np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)


def test_c5_shape_poor_seeds_mass_empties_vs_oracle():
    # c5's defining feature (BASELINE.json configs[4]) at the c5 shape: d=128,
    # k=4096 seeded with 3 data rows + 4093 far-away points, so iteration 1
    # leaves 4093 clusters empty and the takeSample policy
    # (kmeans_spark.py:191-204, seed = the pinned int(time.time())) replaces
    # them; then predict.  Checked against the oracle's restatement of the
    # whole loop (same seed, same policy).
    n, d, k = 12000, 128, 4096
    X = _blobs(n, d, 64, seed=55)
    far = np.full((k - 3, d), 100.0) + np.arange(k - 3)[:, None]
    C0 = np.vstack([X[[0, 1, 2]], far])
    ka = _km()
    seed = 1700000777

    class Pinned(ka.KMeans):
        def _initialize_centroids(self, run):
            return C0.copy()

        def _empty_seed(self):
            return seed

    sc = ka.LocalContext()
    rdd = sc.parallelize(X, 4)
    km = Pinned(k=k, max_iter=2, tolerance=1e-12, compute_sse=True)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        km.fit(rdd, sc)
    lines = []
    ref = orc.lloyd_fit(X, k, 2, 1e-12, 0, True, 4, init_centroids=C0, empty_seed=lambda: seed, log=lines.append)
    assert ref["records"][0]["empty"] and len(ref["records"][0]["empty"]) >= 4000
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
    assert_logs_match(buf.getvalue(), "\n".join(lines) + "\n")
    labels = km.predict(rdd, sc).to_numpy()
    assert _check_labels(X, ref["centroids"], labels) == 0
    assert km._runner.device_repairs >= 1   # replaced on the GPU, inside a batch


@pytest.mark.parametrize("n,d,k,slices,seed", [
    (200_000, 8, 300, 7, 1700000001),     # > 65536 rows: PySpark's sampler over 7 MT19937 streams
    (90_000, 5, 40, 1, 2 ** 40 + 17),     # one partition, a seed above 2^32 (two key words)
    (3000, 3, 2900, 3, 12345),            # ~2900 picks of 3000 rows: 4x-expectation slots, shuffle of ~3000
])
def test_device_empty_repair_matches_takesample_policy(n, d, k, slices, seed):
    # far seeds empty k - 3 clusters on iteration 1; the device replaces them by
    # takeSample(False, k - 3, seed) rows (kmeans_spark.py:191-204) inside the
    # batch; the oracle restates PySpark's takeSample + CPython's random
    X = _blobs(n, d, 8, seed=n + k)
    far = np.full((k - 3, d), 100.0) + np.arange(k - 3)[:, None]
    C0 = np.vstack([X[[0, 1, 2]], far])
    ka = _km()

    class Pinned(ka.KMeans):
        def _initialize_centroids(self, run):
            return C0.copy()

        def _empty_seed(self):
            return seed

    sc = ka.LocalContext()
    rdd = sc.parallelize(X, slices)
    km = Pinned(k=k, max_iter=2, tolerance=1e-12, compute_sse=True)
    km.verbose = False
    km.fit(rdd, sc)
    ref = orc.lloyd_fit(X, k, 2, 1e-12, 0, True, slices, init_centroids=C0, empty_seed=lambda: seed)
    assert len(ref["records"][0]["empty"]) == k - 3
    assert km._runner.device_repairs >= 1
    np.testing.assert_allclose(km.centroids, ref["centroids"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(km.sse_history, ref["sse_history"], rtol=1e-9)
