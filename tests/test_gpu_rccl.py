"""The RCCL path of the per-iteration all-reduce (torch backend "nccl" = RCCL
on ROCm), on the GPU.

One rank: the test box has one GPU, and RCCL does not run two ranks on one
device.  It is still the real multi-rank code path: ``HipEngine(distributed=
True)`` binds the statistics buffer to a torch tensor, ``km_assign_stats``
fills it on the engine stream, ``run_collective(dist.all_reduce)`` runs the
RCCL all-reduce ordered after it and makes the engine stream wait for it
(``work.wait()``, engine.py), and ``km_update`` / ``km_update_async`` read the
result.  A missing order would read a buffer the collective is still writing.
Checked against the oracle (kmeans_spark.py:266-318) over single iterations
and over a batch.
"""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _child(port, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        import kmeans_amd  # noqa: F401  (package alias)
        from kmeans_amd.engine import HipEngine
        from oracle import kmeans_oracle as orc
        rng = np.random.default_rng(5)
        n, d, k = 120_000, 64, 256
        # Gaussian noise (test_b style): no exact convergence within 6 iterations
        X = rng.standard_normal((n, d)).astype(np.float32).astype(np.float64)
        C0 = X[rng.choice(n, k, replace=False)]
        ref = orc.lloyd_fit(X, k, 6, 1e-12, 0, True, 1, init_centroids=C0)
        out = {"backend": dist.get_backend()}
        eng = HipEngine(0, distributed=True)
        eng.load_host(X)
        eng.set_sse(True)
        # three single iterations (km_update: host sync each)
        eng.set_centroids(C0)
        sse = []
        for _ in range(3):
            eng.assign_stats()
            eng.run_collective(dist.all_reduce)
            st, _ = eng.update()
            sse.append(st.sse)
            eng.commit()
        out["single"] = (eng.get_centroids(0), sse)
        # the same three, then three more, as batches (no host sync inside)
        eng.set_centroids(C0)
        sse_b = []
        for m in (3, 3):
            eng.batch_begin()
            for _ in range(m):
                eng.assign_stats()
                eng.run_collective(dist.all_reduce)
                eng.update_async(1e-300, 0)
            recs = eng.batch_end(m)
            assert len(recs) == m, [(st.stop_reason, st.max_shift, st.n_empty) for st, _ in recs]
            sse_b += [st.sse for st, _ in recs]
            eng.commit()
        out["batch"] = (eng.get_centroids(0), sse_b)
        out["ref"] = (ref["centroids"], ref["sse_history"])
        eng.close()
        q.put(out)
    except Exception as e:  # report, do not hang the parent
        q.put({"error": repr(e)})
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_allreduce_ordered_on_engine_stream():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(60)
    assert "error" not in out, out.get("error")
    assert p.exitcode == 0
    assert out["backend"] == "nccl"
    C6, sse6 = out["ref"]
    _, sse_single = out["single"]
    np.testing.assert_allclose(sse_single, sse6[:3], rtol=1e-9)
    C6_batch, sse_batch = out["batch"]
    np.testing.assert_allclose(sse_batch, sse6, rtol=1e-9)
    np.testing.assert_allclose(C6_batch, C6, rtol=1e-9, atol=1e-9)


def _child_repair(port, q):
    # layout mode 2 (rows spread over ranks) driven through RCCL at world 1:
    # the repair rows go through the same stream-ordered all-reduce as on 8
    # GPUs; the c5_poor golden (k = 512, ~509 empty clusters at the first
    # update, reference-generated) must come out exactly
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        import kmeans_amd as ka
        from kmeans_amd.engine import HipEngine
        from conftest import load_golden
        g = load_golden("c5_poor")
        X = g["X"]
        rdd = ka.LocalContext().parallelize(X, int(g["slices"]))
        sizes = [rdd.partition_len(i) for i in range(rdd.getNumPartitions())]
        k, tol, seed = int(g["k"]), float(g["tol"]), int(g["time_seed"])
        eng = HipEngine(0, distributed=True)
        eng.load_host(X)
        eng.set_layout(sizes, 0, 2)
        eng.set_sse(bool(g["sse"]))
        eng.set_centroids(g["init"])
        sse, it, repaired, waited = [], 0, 0, 0
        max_iter = int(g["max_iter"])
        while it < max_iter:
            m = min(4, max_iter - it)
            eng.repair_bind()
            eng.batch_begin()
            for _ in range(m):
                eng.assign_stats()
                eng.run_collective(dist.all_reduce)
                eng.update_async(tol, seed)
                if eng.repair_state()[1]:
                    waited += 1
                    eng.repair_exchange(dist.all_reduce)
            recs = eng.batch_end(m)
            for st, _ in recs:
                sse.append(st.sse)
                repaired += int(st.repaired)
            it += len(recs)
            last = recs[-1][0]
            assert last.stop_reason != 2, "empty stop: the device repair did not run"
            eng.commit()
            if last.stop_reason == 1:
                break
        q.put({"C": eng.get_centroids(0), "sse": sse, "repaired": repaired, "waited": waited,
               "ref": (g["centroids"], g["sse_history"])})
        eng.close()
    except Exception as e:  # report, do not hang the parent
        q.put({"error": repr(e)})
        raise
    finally:
        dist.destroy_process_group()


def test_rccl_device_repair_with_rows_over_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_child_repair, args=(_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(60)
    assert "error" not in out, out.get("error")
    assert p.exitcode == 0
    assert out["repaired"] > 0 and out["waited"] > 0
    C, sse = out["ref"]
    np.testing.assert_allclose(out["sse"], sse, rtol=1e-9)
    np.testing.assert_allclose(out["C"], C, rtol=1e-9, atol=1e-9)
