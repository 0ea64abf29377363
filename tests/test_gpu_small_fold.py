"""The small path's one-launch iteration (k_assign_small with the update
folded into its last workgroup) against the two-launch form, and every call
that must flush a deferred assign.

kmeans_spark.py:147-206: assign + reduceByKey + update.  On the small path
(k <= 32, dp <= 64) inside a batch on one rank, km_assign_stats defers its
launch and km_update_async launches assign + update as one kernel; rows the
fp32 bound cannot settle queue per wave in LDS (32 per wave) and beyond that
in a global queue the last workgroup drains.  Binding an external statistics
buffer turns the fold off (a caller may reduce the buffer between the two
calls), so the same iterations run once folded and once unfolded here, on
input where half of the rows tie exactly between two centroids (queued, far
more than 32 per wave): labels, centroids, counts, SSE and the queue counts
must be identical, and equal to the oracle.
"""
import ctypes

import numpy as np
import pytest

from oracle import kmeans_oracle as orc

pytestmark = pytest.mark.gpu


def _engine():
    from kmeans_amd.comm import Communicator
    from kmeans_amd.engine import make_engine
    return make_engine(Communicator())


def _tie_data(n=2_000_000, d=16, seed=7):
    # 4 blobs, each with a centroid pair m +- e_0: half of the rows have
    # x_0 = m_0 exactly, so (x_0 - c_0)^2 = 1 for both centroids of the pair
    # -- an exact float64 tie (np.argmin keeps the lower index) that no fp32
    # bound separates: every such row queues in the first iteration (about
    # 250 per wave at this n, far past the 32 the wave's LDS queue holds);
    # the other half keeps both clusters of each pair non-empty
    rng = np.random.default_rng(seed)
    m = rng.uniform(-5, 5, (4, d)).astype(np.float32).astype(np.float64)
    blob = rng.integers(0, 4, n)
    noise = 0.5 * rng.standard_normal((n, d))
    noise[: n // 2, 0] = 0.0
    X = (m[blob] + noise).astype(np.float32).astype(np.float64)
    e0 = np.zeros(d)
    e0[0] = 1.0
    C0 = np.concatenate([m + e0, m - e0])
    return X, C0


def _run(X, C0, iters, external):
    import torch
    eng = _engine()
    eng.load_host(X.astype(np.float32))
    eng.set_sse(True)
    eng.set_centroids(C0)
    k, d = C0.shape
    keep = None
    if external:
        keep = torch.zeros(k * (d + 1) + 1, dtype=torch.float64, device="cuda:0")
        torch.cuda.synchronize()
        rc = eng.lib.km_bind_stats_buffer(eng.ctx, ctypes.c_void_p(keep.data_ptr()))
        assert rc == 0
    eng.batch_begin()
    for _ in range(iters):
        eng.assign_stats()
        eng.update_async(1e-300, 0)
    recs = eng.batch_end(iters)
    out = {"labels": eng.labels(), "C": eng.get_centroids(0), "counts": [r[1].copy() for r in recs],
           "sse": [r[0].sse for r in recs], "q": [(r[0].q_rerank, r[0].q_full) for r in recs], "ran": len(recs)}
    del keep
    return out


def test_small_path_fold_equals_two_launches_with_global_queue():
    X, C0 = _tie_data()
    a = _run(X, C0, 3, external=False)
    b = _run(X, C0, 3, external=True)
    assert a["ran"] == b["ran"] == 3
    # the tied half queued in the first iteration: the per-wave LDS queue
    # (32) overflows into the global queue the last workgroup drains
    assert a["q"][0][0] + a["q"][0][1] >= len(X) // 2
    assert a["q"] == b["q"]
    np.testing.assert_array_equal(a["labels"], b["labels"])
    for ca, cb in zip(a["counts"], b["counts"]):
        np.testing.assert_array_equal(ca, cb)
    np.testing.assert_allclose(a["C"], b["C"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(a["sse"], b["sse"], rtol=1e-12)
    ref = orc.lloyd_fit(X, len(C0), 3, 1e-300, 0, True, 1, init_centroids=C0)
    np.testing.assert_allclose(a["sse"], ref["sse_history"], rtol=1e-9)
    # the committed centroids after three iterations (the batch's speculative
    # commit of the last one is the state km_batch_end leaves before commit)
    C2 = orc.lloyd_fit(X, len(C0), 2, 1e-300, 0, True, 1, init_centroids=C0)["centroids"]
    np.testing.assert_array_equal(a["labels"], orc.assign(X, C2)[0])


@pytest.mark.parametrize("between", ["labels", "stats_buffer", "sync", "get_centroids", "set_sse"])
def test_flush_points_between_assign_and_update(between):
    # a deferred assign (fold pending) followed by a call that must launch it
    # first; the iteration then completes with the usual update launch
    X, C0 = _tie_data(n=200_000)
    eng = _engine()
    eng.load_host(X.astype(np.float32))
    eng.set_sse(True)
    eng.set_centroids(C0)
    eng.batch_begin()
    eng.assign_stats()
    if between == "labels":
        np.testing.assert_array_equal(eng.labels(), orc.assign(X, C0)[0])
    elif between == "stats_buffer":
        p, n = ctypes.c_void_p(), ctypes.c_int64()
        assert eng.lib.km_stats_buffer(eng.ctx, ctypes.byref(p), ctypes.byref(n)) == 0
    elif between == "sync":
        eng.sync()
    elif between == "get_centroids":
        np.testing.assert_array_equal(eng.get_centroids(0), C0)
    elif between == "set_sse":
        eng.set_sse(True)
    eng.update_async(1e-300, 0)
    recs = eng.batch_end(1)
    assert len(recs) == 1
    ref = orc.lloyd_fit(X, len(C0), 1, 1e-300, 0, True, 1, init_centroids=C0)
    np.testing.assert_allclose(recs[0][0].sse, ref["sse_history"][0], rtol=1e-9)
    np.testing.assert_array_equal(eng.labels(), orc.assign(X, C0)[0])
    np.testing.assert_allclose(eng.get_centroids(1), ref["centroids"], rtol=1e-9, atol=1e-12)


def test_serpentine_sweeps_agree():
    # k_assign_small sweeps the rows last-first on every other launch (the
    # Infinity Cache then serves the previous sweep's tail): two consecutive
    # launches on the same centroids, one in each direction, must give the
    # oracle's labels, identical counts and sums equal up to float64
    # summation order
    import torch
    X, C0 = _tie_data(n=1_000_000)
    k, d = C0.shape
    eng = _engine()
    eng.load_host(X.astype(np.float32))
    eng.set_sse(True)
    eng.set_centroids(C0)
    keep = torch.zeros(k * (d + 1) + 1, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    assert eng.lib.km_bind_stats_buffer(eng.ctx, ctypes.c_void_p(keep.data_ptr())) == 0
    ref_labels, ref_mind, _ = orc.assign(X, C0)
    outs = []
    for _ in range(2):
        eng.assign_stats()
        eng.sync()
        outs.append((eng.labels(), keep.cpu().numpy().copy()))
    (la, sa), (lb, sb) = outs
    np.testing.assert_array_equal(la, ref_labels)
    np.testing.assert_array_equal(lb, ref_labels)
    t_a, t_b = sa[:-1].reshape(k, d + 1), sb[:-1].reshape(k, d + 1)
    np.testing.assert_array_equal(t_a[:, d], t_b[:, d])
    np.testing.assert_array_equal(t_a[:, d], np.bincount(ref_labels, minlength=k))
    np.testing.assert_allclose(t_b[:, :d], t_a[:, :d], rtol=1e-12, atol=1e-9)
    sums = np.zeros((k, d))
    np.add.at(sums, ref_labels, X)
    np.testing.assert_allclose(t_a[:, :d], sums, rtol=1e-9, atol=1e-6)
    np.testing.assert_allclose([sa[-1], sb[-1]], (ref_mind ** 2).sum(), rtol=1e-9)
    del keep
