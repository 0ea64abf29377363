"""Multi-rank path on the GPU: two processes (torch.distributed over gloo, both
on cuda:0 because the test box has one GPU) run the real HIP engine on their
row shards and exchange the [k][d+1] float64 statistics with the same
stream-ordered all-reduce the RCCL path uses (engine.run_collective).  Results
must match the reference's golden vectors like the single-rank run does:
the shard-invariance the 1..8 GPU scaling bench relies on
(kmeans_spark.py:169-173 -> one all-reduce per iteration)."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, name, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import contextlib
        import io
        import kmeans_amd as ka
        from conftest import load_golden
        g = load_golden(name)
        init = g["init"]

        class Pinned(ka.KMeans):
            def _initialize_centroids(self, run):
                return init.copy()

            def _empty_seed(self):
                return int(g["time_seed"])

        sc = ka.LocalContext()
        rdd = sc.parallelize(g["X"], int(g["slices"]))
        km = Pinned(k=int(g["k"]), max_iter=int(g["max_iter"]), tolerance=float(g["tol"]), seed=int(g["seed"]),
                    compute_sse=bool(g["sse"]))
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            km.fit(rdd, sc)
        pred = km.predict(rdd, sc)
        # collect(): to the driver (rank 0) only; everywhere=True: every rank
        labels = (np.array(pred.collect()), np.array(pred.collect(everywhere=True)))
        assert km._runner.engine.distributed
        assert km._runner.device_repair == 2
        q.put((rank, km.centroids, km.sse_history, labels, buf.getvalue(), km._runner.pl.n_local,
               km._runner.device_repairs))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e), None, None, None, None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["test_a", "empty", "c3_small", "c5_poor"])
def test_two_ranks_on_gpu_match_reference(golden, name):
    # "empty" and "c5_poor" (k = 512, ~509 empty clusters at the first update)
    # repair their empty clusters on the devices of both ranks (layout mode 2:
    # same picks on every rank, rows from their owners through one
    # stream-ordered all-reduce), with no host round trip
    import torch.multiprocessing as mp
    g = golden(name)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=110) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0, res
    assert sum(r[5] for r in res) == len(g["X"])  # the shards partition the rows
    for rank, C, sse, labels, out, _, reps in res:
        np.testing.assert_allclose(C, g["centroids"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(sse, g["sse_history"], rtol=1e-9)
        np.testing.assert_array_equal(labels[0], g["labels"] if rank == 0 else g["labels"][:0])
        np.testing.assert_array_equal(labels[1], g["labels"])
        if name in ("empty", "c5_poor"):
            assert reps > 0, "the empty clusters were not repaired on the device"
    assert res[0][4] and not res[1][4]  # only rank 0 logs


def _rank_delta(rank, world, port, q):
    # c3 geometry (d 64, k 256), compute_sse off: from the second iteration
    # every rank runs k_s1 with delta statistics, and the all-reduce sums the
    # ranks' deltas, which k_s1_apply folds into each rank's copy of the full
    # sums (the same on every rank: they were all-reduced too)
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import kmeans_amd as ka
        X, C0 = _delta_data()

        class Pinned(ka.KMeans):
            def _initialize_centroids(self, run):
                return C0.copy()

            def _empty_seed(self):
                return 1234

        km = Pinned(k=len(C0), max_iter=6, tolerance=1e-12, compute_sse=False)
        km.verbose = False
        km.fit(X)
        eng = km._runner.engine
        q.put((rank, km.centroids, eng.screen(), km._runner.last["counts"].copy(), km._runner.iterations_run
               if hasattr(km._runner, "iterations_run") else None))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def _delta_data():
    rng = np.random.default_rng(91)
    C = rng.uniform(-10, 10, (256, 64))
    X = (C[rng.integers(0, 256, 40000)] + rng.standard_normal((40000, 64))).astype(np.float32).astype(np.float64)
    C0 = X[np.random.default_rng(92).choice(len(X), 256, replace=False)]
    return X, C0


def test_two_ranks_delta_statistics_c3_shape():
    import torch.multiprocessing as mp
    from oracle import kmeans_oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_delta, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=110) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0, res
    X, C0 = _delta_data()
    ref = orc.lloyd_fit(X, 256, 6, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: 1234)
    for rank, C, screen, counts, _ in res:
        assert screen == 4, "k_s1 (delta statistics) not selected"
        np.testing.assert_allclose(C, ref["centroids"], rtol=1e-9, atol=1e-9)
        assert int(counts.sum()) == len(X)


def _rank_uneven(rank, world, port, d, k, q):
    # rank 0 holds all rows but 500, rank 1 the last 500: their k_s1 grids
    # differ (rank 1 fills a few workgroups), and both must still make the
    # same delta / full choice, or the all-reduce would add one rank's deltas
    # to the other's full sums
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import kmeans_amd as ka
        from kmeans_amd import dataset
        X, C0 = _uneven_data(d, k)
        dataset.rank_rows = lambda n, w, r: (0, n - 500) if r == 0 else (n - 500, n)

        class Pinned(ka.KMeans):
            def _initialize_centroids(self, run):
                return C0.copy()

            def _empty_seed(self):
                return 1234

        km = Pinned(k=k, max_iter=5, tolerance=1e-12, compute_sse=False)
        km.verbose = False
        km.fit(X)
        eng = km._runner.engine
        q.put((rank, km.centroids, eng.info()["delta_stats"], km._runner.pl.n_local, km._runner.last["counts"].copy()))
    except Exception as e:  # surface the failure in the parent
        q.put((rank, repr(e), None, None, None))
        raise
    finally:
        dist.destroy_process_group()


def _uneven_data(d, k):
    rng = np.random.default_rng(95 + d)
    C = rng.uniform(-10, 10, (300, d))
    X = (C[rng.integers(0, 300, 20000)] + rng.standard_normal((20000, d))).astype(np.float32).astype(np.float64)
    C0 = X[np.random.default_rng(96).choice(len(X), k, replace=False)]
    return X, C0


@pytest.mark.parametrize("d,k,delta", [
    (18, 1000, 1),   # dp 32, kp 1024: the LDS delta table fits for any grid on both ranks
    (19, 1000, 1),   # fits only beside a small grid's wave prefix: the fold's range count may differ by rank, the deltas do not
])
def test_two_ranks_uneven_shards_same_statistics_mode(d, k, delta):
    import torch.multiprocessing as mp
    from oracle import kmeans_oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_uneven, args=(r, 2, port, d, k, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=110) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0, res
    X, C0 = _uneven_data(d, k)
    assert [r[3] for r in res] == [len(X) - 500, 500]
    ref = orc.lloyd_fit(X, k, 5, 1e-12, 0, False, 1, init_centroids=C0, empty_seed=lambda: 1234)
    for rank, C, dstat, _, counts in res:
        assert dstat == delta, (rank, dstat)
        np.testing.assert_allclose(C, ref["centroids"], rtol=1e-9, atol=1e-9)
        assert int(counts.sum()) == len(X)
