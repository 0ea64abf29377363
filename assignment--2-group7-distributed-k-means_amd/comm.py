"""Collectives of the Lloyd loop over ``torch.distributed`` (one process per GPU).

The reference moves data with Spark (kmeans_spark.py): ``sc.broadcast`` of the
centroids (L268), the ``reduceByKey`` shuffle + ``collect`` of per-cluster
partial sums (L169-173) and the ``.sum()`` of partition SSEs (L237).  Here:

* every rank holds the same centroids and recomputes the same update, so
  there is no broadcast;
* the only per-iteration exchange is ONE sum all-reduce of the float64
  ``[k][d+1] + 1`` statistics buffer (per-cluster sums and counts, plus the
  SSE slot: every row's float64 residual to its centroid), issued by
  ``allreduce_stats`` on the device buffer itself, ordered on the engine's
  stream (``HipEngine.run_collective``; backend ``nccl`` = RCCL over xGMI on
  MI355X; ``gloo`` on CPU for tests);
* a few host-side values (data moments at load time, replacement rows on the
  rare empty-cluster path, the wall-clock seed, predictions) use the small
  helpers below.

With no process group (or world size 1) every call is a local no-op.
"""
from __future__ import annotations

import os
from typing import Any, List

import numpy as np


def _dist():
    try:
        import torch.distributed as dist
    except Exception:  # torch absent: single process only
        return None
    if dist.is_available() and dist.is_initialized():
        return dist
    return None


class Communicator:
    def __init__(self):
        self.dist = _dist()
        if self.dist is None:
            self.rank, self.world = 0, 1
            self.backend = None
        else:
            self.rank = self.dist.get_rank()
            self.world = self.dist.get_world_size()
            self.backend = self.dist.get_backend()

    @property
    def local_rank(self) -> int:
        return int(os.environ.get("LOCAL_RANK", self.rank if self.world > 1 else 0))

    def _tensor(self, arr: np.ndarray):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(arr))
        if self.backend == "nccl":
            t = t.to(f"cuda:{self.local_rank}")
        return t

    # -- host-array collectives ----------------------------------------------
    def allreduce_np(self, arr) -> np.ndarray:
        arr = np.asarray(arr)
        if self.world == 1:
            return arr.copy()
        t = self._tensor(arr)
        self.dist.all_reduce(t)
        return t.cpu().numpy()

    def allgather_int(self, v: int) -> List[int]:
        if self.world == 1:
            return [int(v)]
        t = self._tensor(np.array([v], dtype=np.int64))
        out = [t.clone() for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [int(x.cpu().item()) for x in out]

    def broadcast_obj(self, obj: Any, src: int = 0) -> Any:
        if self.world == 1:
            return obj
        lst = [obj if self.rank == src else None]
        self.dist.broadcast_object_list(lst, src=src)
        return lst[0]

    def allgather_array(self, arr: np.ndarray) -> List[np.ndarray]:
        """Variable-length all-gather of 1-D arrays (predict results)."""
        if self.world == 1:
            return [np.asarray(arr)]
        arr = np.ascontiguousarray(arr)
        sizes = self.allgather_int(arr.shape[0])
        m = max(sizes) if sizes else 0
        pad = np.zeros(max(m, 1), dtype=arr.dtype)
        pad[:arr.shape[0]] = arr
        t = self._tensor(pad)
        out = [t.clone() for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [o.cpu().numpy()[:s] for o, s in zip(out, sizes)]

    def gather_array(self, arr: np.ndarray, root: int = 0):
        """Variable-length gather of 1-D arrays to ``root``: the list of every
        rank's array there, None on the other ranks (predict results to the
        driver, as Spark's collect())."""
        if self.world == 1:
            return [np.asarray(arr)]
        arr = np.ascontiguousarray(arr)
        sizes = self.allgather_int(arr.shape[0])
        m = max(sizes) if sizes else 0
        pad = np.zeros(max(m, 1), dtype=arr.dtype)
        pad[:arr.shape[0]] = arr
        t = self._tensor(pad)
        out = [t.clone() for _ in range(self.world)] if self.rank == root else None
        self.dist.gather(t, out, dst=root)
        return [o.cpu().numpy()[:s] for o, s in zip(out, sizes)] if self.rank == root else None

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    # -- the per-iteration exchange -------------------------------------------
    def allreduce_stats(self, engine) -> None:
        """Sum the per-rank partial statistics (reduceByKey + collect, L169-173)."""
        if self.world == 1:
            return
        engine.run_collective(self.dist.all_reduce)
