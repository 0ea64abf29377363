"""Inputs of ``fit(rdd, sc)`` / ``predict(rdd, sc)`` and their placement.

The reference receives a PySpark RDD of ``(d,)`` float arrays built by
``sc.parallelize(X[, numSlices]).cache()`` (kmeans_spark.py:369, 418, 471,
518, 568).  This module accepts, duck-typed:

* ``LocalRDD`` — this package's stand-in for such an RDD
  (``LocalContext().parallelize(X, numSlices)`` mirrors ``sc.parallelize``),
* a real PySpark RDD (anything with ``glom().collect()``),
* a NumPy array ``[n][d]`` (one partition),
* ``DeviceBlobs`` — a synthetic Gaussian-blob dataset generated directly in
  HBM (benchmarks; nothing on the host).

``place`` turns one into a ``Placement``: the global partition layout (needed
by the takeSample policy), this rank's contiguous block of partitions and
rows, and how to fetch rows by global index.  With W ranks, rank r owns
partitions ``[r*P//W, (r+1)*P//W)`` (an array input is cut into W row blocks),
so concatenating the ranks' predictions restores input order.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, List, Optional, Sequence

import numpy as np


class Broadcast:
    def __init__(self, value):
        self.value = value

    def unpersist(self, blocking=False):
        pass


class LocalRDD:
    """Partitioned rows held in host memory (the RDD slot of the reference)."""

    def __init__(self, partitions: Sequence[Any], ctx: Optional["LocalContext"] = None):
        self._parts = list(partitions)
        self.ctx = ctx

    def cache(self):
        return self

    def persist(self, *a, **kw):
        return self

    def unpersist(self, blocking=False):
        return self

    def getNumPartitions(self) -> int:
        return len(self._parts)

    def glom(self):
        return LocalRDD([[list(p)] for p in self._parts], self.ctx)

    def partition_arrays(self) -> List[np.ndarray]:
        out = []
        for p in self._parts:
            if isinstance(p, np.ndarray) and p.ndim == 2:
                out.append(p)
            else:
                items = list(p)
                out.append(np.asarray(items) if items else None)
        return out

    def collect(self) -> list:
        out = []
        for p in self._parts:
            if isinstance(p, np.ndarray) and p.ndim == 2:
                out.extend(list(p))
            elif isinstance(p, np.ndarray):
                out.extend(p.tolist())
            else:
                out.extend(list(p))
        return out

    def count(self) -> int:
        return sum(len(p) for p in self._parts)

    def repartition(self, n: int) -> "LocalRDD":
        arrs = [a for a in self.partition_arrays() if a is not None]
        X = np.concatenate(arrs) if arrs else np.zeros((0, 0))
        return LocalContext(n).parallelize(X, n)

    def mapPartitions(self, f) -> "LocalRDD":
        return LocalRDD([list(f(iter(p))) for p in self._parts], self.ctx)


class LocalContext:
    """The ``sc`` slot: ``parallelize`` cuts contiguous slices like PySpark."""

    def __init__(self, defaultParallelism: int = 1, appName: Optional[str] = None):
        self.defaultParallelism = defaultParallelism
        self.appName = appName

    def parallelize(self, c, numSlices: Optional[int] = None, numPartitions: Optional[int] = None) -> LocalRDD:
        n_slices = numSlices or numPartitions or self.defaultParallelism
        if isinstance(c, np.ndarray) and c.ndim == 2:
            n = c.shape[0]
            parts = [c[(i * n) // n_slices:((i + 1) * n) // n_slices] for i in range(n_slices)]
        else:
            data = list(c)
            n = len(data)
            parts = [data[(i * n) // n_slices:((i + 1) * n) // n_slices] for i in range(n_slices)]
        return LocalRDD(parts, self)

    def broadcast(self, value):
        return Broadcast(value)

    def setLogLevel(self, level):
        pass

    def stop(self):
        pass


@dataclass
class DeviceBlobs:
    """Synthetic Gaussian blobs (centers uniform in (-box, box), std ``std``)
    generated in HBM by a counter-based generator keyed on the global row, so
    the data are identical for any sharding.  ``n`` is the GLOBAL row count;
    ``partitions`` is the dataset's partition layout for ``takeSample`` (like
    ``sc.parallelize(X, partitions)``), independent of how many GPUs hold it,
    so the initial centroids and the whole run are the same on 1..8 GPUs; the
    Bernoulli pass runs one GPU wave per partition (km_bernoulli_sample)."""
    n: int
    d: int
    n_centers: int
    box: float = 10.0
    std: float = 1.0
    seed: int = 0
    partitions: int = 256


@dataclass
class Placement:
    global_sizes: List[int]          # rows per global partition (takeSample layout)
    local_rows: Optional[np.ndarray]  # this rank's rows (host), None for DeviceBlobs
    row0: int                        # global index of this rank's first row
    n_local: int
    n_global: int
    d: int
    dtype: Any
    host_partitions: Optional[List[np.ndarray]] = field(default=None, repr=False)
    blobs: Optional[DeviceBlobs] = None

    def host_rows(self, gidx: Sequence[int]) -> Optional[np.ndarray]:
        """Rows by global index when every rank holds the data on the host."""
        if self.host_partitions is None:
            return None
        starts = np.cumsum([0] + [len(p) if p is not None else 0 for p in self.host_partitions])
        out = []
        for g in gidx:
            pi = int(np.searchsorted(starts, g, side="right") - 1)
            out.append(self.host_partitions[pi][g - starts[pi]])
        return np.asarray(out, dtype=self.dtype).reshape(len(out), self.d)


def _partitions_of(rdd) -> List[np.ndarray]:
    if isinstance(rdd, np.ndarray):
        if rdd.ndim != 2:
            raise ValueError("input array must be 2-D [n][d]")
        return [rdd]
    if isinstance(rdd, LocalRDD):
        parts = rdd.partition_arrays()
    elif hasattr(rdd, "glom"):  # PySpark RDD (duck-typed)
        parts = [np.asarray(p) if len(p) else None for p in rdd.glom().collect()]
    else:
        raise TypeError(f"unsupported dataset type {type(rdd).__name__}: expected an RDD, LocalRDD, "
                        f"ndarray or DeviceBlobs")
    return parts


def place(rdd, comm) -> Placement:
    if isinstance(rdd, DeviceBlobs):
        W, r = comm.world, comm.rank
        sizes = [((i + 1) * rdd.n) // W - (i * rdd.n) // W for i in range(W)]
        row0 = (r * rdd.n) // W
        P = max(1, int(rdd.partitions))
        layout = [((i + 1) * rdd.n) // P - (i * rdd.n) // P for i in range(P)]
        return Placement(global_sizes=layout, local_rows=None, row0=row0, n_local=sizes[r], n_global=rdd.n,
                         d=rdd.d, dtype=np.float64, blobs=rdd)
    parts = _partitions_of(rdd)
    d = None
    dtype = None
    for p in parts:
        if p is not None and p.size:
            if p.ndim != 2:
                p = p.reshape(len(p), -1)
            d = p.shape[1]
            dtype = p.dtype
            break
    if d is None:
        raise ValueError("Not enough data points (0) to initialize clusters")
    parts = [None if p is None else np.asarray(p).reshape(len(p), d) for p in parts]
    if not np.issubdtype(dtype, np.floating):
        dtype = np.float64
    sizes = [0 if p is None else len(p) for p in parts]
    W, r = comm.world, comm.rank
    if len(parts) == 1 and W > 1:
        # a single array: cut it into W row blocks
        X = parts[0]
        n = len(X)
        parts = [X[(i * n) // W:((i + 1) * n) // W] for i in range(W)]
        mine = [parts[r]]
        row0 = (r * n) // W
        global_sizes = sizes  # the takeSample layout is still ONE partition
        host_parts = [X]
    else:
        P = len(parts)
        lo, hi = (r * P) // W, ((r + 1) * P) // W
        mine = [p for p in parts[lo:hi] if p is not None]
        row0 = int(sum(sizes[:lo]))
        global_sizes = sizes
        host_parts = parts
    local = np.concatenate(mine) if mine else np.zeros((0, d))
    return Placement(global_sizes=global_sizes, local_rows=local, row0=row0, n_local=len(local),
                     n_global=int(sum(sizes)), d=d, dtype=dtype, host_partitions=host_parts)
