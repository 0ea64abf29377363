"""GPU parity at BASELINE.json's full single-GPU sizes, through properties that
do not need the oracle to process every row:

* counts: the per-cluster counts of the statistics pass sum to N and equal the
  histogram of the labels it wrote;
* checksum of checksums: sum_j n_j * c'_j (new centroids times counts, i.e. the
  reduceByKey sums of kmeans_spark.py:169-188) equals sum_i x_i from an
  independent float64 reduction of X;
* cross-path idempotence: predict (the assign kernel without statistics,
  kmeans_spark.py:343-350) returns exactly the labels of the fused
  assign + statistics pass for the same centroids;
* sampled labels: a seeded sample of rows, labelled by the oracle's restatement
  of np.argmin(np.linalg.norm(C - x, axis=1)) (kmeans_spark.py:153-156),
  bit-identical.

c3 = N=100M, d=64, k=256 (the bench workload); c5 = N=50M, d=128, k=4096
(one GPU holding all of it; the unfused MFMA path, chunked centroids, label-sort
statistics); c4 = N=1B, d=32, k=1024 (128 GB resident on one GPU: 64-bit row
indexing, statistics tiled over feature ranges).
"""
import numpy as np
import pytest

from oracle import kmeans_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,d,k,centers,sample,chunk", [
    (100_000_000, 64, 256, 256, 20000, 1024),      # c3
    (50_000_000, 128, 4096, 4096, 3000, 48),       # c5
    (1_000_000_000, 32, 1024, 1024, 3000, 256),    # c4: 128 GB of rows on one GPU
])
def test_full_size_properties(N, d, k, centers, sample, chunk):
    import kmeans_amd
    from kmeans_amd.comm import Communicator

    km = kmeans_amd.KMeans(k=k, max_iter=1, tolerance=1e-12, seed=42, compute_sse=True)
    km.verbose = False
    data = kmeans_amd.DeviceBlobs(n=N, d=d, n_centers=centers, box=10.0, std=1.0, seed=2024)
    run = km._make_runner(data, Communicator())
    eng = run.engine
    C0 = km._initialize_centroids(run)
    eng.set_centroids(C0)
    eng.set_sse(True)
    sx = eng.sum_x()

    eng.assign_stats()
    st, counts = eng.update()
    C1 = eng.get_centroids(1)
    labels = eng.labels()
    assert labels.shape == (N,)
    assert labels.min() >= 0 and labels.max() < k

    assert int(counts.sum()) == N
    np.testing.assert_array_equal(np.bincount(labels, minlength=k), counts)

    nz = counts > 0
    tot = (counts[nz, None].astype(np.float64) * C1[nz]).sum(axis=0)
    # |x| <= ~15 per feature: float64 sums of 1e8 such values agree to ~1e-7
    np.testing.assert_allclose(tot, sx, rtol=1e-9, atol=1e-3)

    pred = eng.predict()                      # current centroids are still C0
    np.testing.assert_array_equal(pred, labels)

    gidx = np.sort(np.random.default_rng(7).choice(N, sample, replace=False))
    Xs = run.rows(gidx.tolist())
    lab_ref, _, _ = orc.assign(np.asarray(Xs, dtype=np.float64), C0, chunk=chunk)
    np.testing.assert_array_equal(labels[gidx], lab_ref)
    assert np.isfinite(st.sse) and st.sse > 0
    # the sampled rows' own residuals (float64, oracle distances) scaled to N
    # bracket the SSE loosely: blobs of std 1, so ~d per row
    _, mind, _ = orc.assign(np.asarray(Xs, dtype=np.float64), C0, chunk=chunk)
    est = float(np.sum(mind ** 2)) * N / sample
    assert 0.8 * est < st.sse < 1.25 * est, (st.sse, est)


def test_full_size_c5_poor_seeds_device_repair():
    # c5 at full size (50M x 128, k = 4096) seeded with 3 data rows + 4093 far
    # points: one iteration empties 4093 clusters, which the device replaces
    # inside the batch.  The replacement rows must be exactly the rows that
    # the host restatement of takeSample(False, 4093, seed) picks
    # (kmeans_spark.py:191-204; PySpark over the dataset's 256 partitions).
    import kmeans_amd
    from kmeans_amd import sampling
    from kmeans_amd.comm import Communicator

    N, d, k, seed = 50_000_000, 128, 4096, 1700000999

    class Pinned(kmeans_amd.KMeans):
        def _empty_seed(self):
            return seed

    km = Pinned(k=k, max_iter=1, tolerance=1e-12, seed=42, compute_sse=True)
    km.verbose = False
    data = kmeans_amd.DeviceBlobs(n=N, d=d, n_centers=k, box=10.0, std=1.0, seed=2024)
    run = km._make_runner(data, Communicator())
    eng = run.engine
    C0 = np.vstack([km._initialize_centroids(run)[:3], np.full((k - 3, d), 100.0) + np.arange(k - 3)[:, None]])
    eng.set_centroids(C0)
    eng.set_sse(True)
    run.run(km, None, 1)
    assert run.device_repairs == 1
    counts = run.last["counts"]
    empty = np.nonzero(counts == 0)[0]
    assert len(empty) >= 4000 and int(counts.sum()) == N
    C1 = eng.get_centroids(0)
    gidx = sampling.take_sample(run.pl.global_sizes, len(empty), seed)
    np.testing.assert_array_equal(C1[empty], run.rows(gidx[:len(empty)]))
    full = np.nonzero(counts > 0)[0]
    assert np.all(np.isfinite(C1[full])) and np.all(np.abs(C1[full]) < 20)


def test_full_size_c2_through_lloyd_runner():
    # c2 (10M x 16, k 8) through LloydRunner.run on one rank: the small path's
    # one-launch iteration (k_assign_small with the update folded into its
    # last workgroup, which takes the queued rows over from the others) at
    # full size.  Iterations 1-2, then 3 alone, so the centroids the third
    # assignment used are known: counts, checksum of checksums and sampled
    # labels of that assignment (kmeans_spark.py:147-206).
    import kmeans_amd
    from kmeans_amd.comm import Communicator

    N, d, k = 10_000_000, 16, 8
    km = kmeans_amd.KMeans(k=k, max_iter=10, tolerance=1e-300, seed=42)
    km.verbose = False
    data = kmeans_amd.DeviceBlobs(n=N, d=d, n_centers=k, box=10.0, std=1.0, seed=2024)
    run = km._make_runner(data, Communicator())
    eng = run.engine
    eng.set_centroids(km._initialize_centroids(run))
    assert eng.info()["path"] == 1
    sx = eng.sum_x()
    run.run(km, None, 2)
    assert run.iterations_ran == 2
    C_prev = eng.get_centroids(0)
    run.run(km, None, 3, first=2)
    assert run.iterations_ran == 3
    counts = np.asarray(run.last["counts"])
    C3 = eng.get_centroids(0)
    labels = eng.labels()
    assert int(counts.sum()) == N
    np.testing.assert_array_equal(np.bincount(labels, minlength=k), counts)
    nz = counts > 0
    tot = (counts[nz, None].astype(np.float64) * C3[nz]).sum(axis=0)
    np.testing.assert_allclose(tot, sx, rtol=1e-9, atol=1e-4)
    gidx = np.sort(np.random.default_rng(11).choice(N, 20000, replace=False))
    Xs = np.asarray(run.rows(gidx.tolist()), dtype=np.float64)
    lab_ref, _, _ = orc.assign(Xs, C_prev)
    np.testing.assert_array_equal(labels[gidx], lab_ref)
    # the update of the same launch: the new centroids are the sampled
    # clusters' means to within the sample's noise, and exactly the folded
    # sums over the counts (checked above); predict with them is stable
    pred = eng.predict()
    np.testing.assert_array_equal(pred[gidx], orc.assign(Xs, C3)[0])


def test_full_size_c3_delta_fit_through_lloyd_runner():
    # the kernel the bench times (BASELINE metric, c3 = 100M x 64, k 256,
    # compute_sse off): k_s1<2, 8, 1> with delta statistics (k_s1_delta, then
    # k_s1_apply folding the changes into the kept full sums) at full size,
    # through LloydRunner.run as fit drives it (kmeans_spark.py:147-206).
    # Iterations 1-5 (the first with full statistics, then four delta passes),
    # then iteration 6 alone so its input centroids are known: the counts are
    # the label histogram, sum_j n_j c_j equals an independent float64 sum of X
    # (the full sums after five rounds of deltas), and 20k sampled labels are
    # the oracle's
    import kmeans_amd
    from kmeans_amd.comm import Communicator

    N, d, k = 100_000_000, 64, 256
    km = kmeans_amd.KMeans(k=k, max_iter=10, tolerance=1e-300, seed=42)
    km.verbose = False
    data = kmeans_amd.DeviceBlobs(n=N, d=d, n_centers=k, box=10.0, std=1.0, seed=2024)
    run = km._make_runner(data, Communicator())
    eng = run.engine
    eng.set_centroids(km._initialize_centroids(run))
    sx = eng.sum_x()
    run.run(km, None, 5)
    assert run.iterations_ran == 5
    assert eng.screen() == 4 and eng.info()["delta_stats"] == 1
    C_prev = eng.get_centroids(0)
    run.run(km, None, 6, first=5)
    assert run.iterations_ran == 6 and eng.info()["delta_stats"] == 1
    counts = np.asarray(run.last["counts"])
    C6 = eng.get_centroids(0)
    labels = eng.labels()
    assert int(counts.sum()) == N
    np.testing.assert_array_equal(np.bincount(labels, minlength=k), counts)
    nz = counts > 0
    tot = (counts[nz, None].astype(np.float64) * C6[nz]).sum(axis=0)
    np.testing.assert_allclose(tot, sx, rtol=1e-9, atol=1e-3)
    gidx = np.sort(np.random.default_rng(13).choice(N, 20000, replace=False))
    Xs = np.asarray(run.rows(gidx.tolist()), dtype=np.float64)
    np.testing.assert_array_equal(labels[gidx], orc.assign(Xs, C_prev, chunk=1024)[0])
