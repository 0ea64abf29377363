"""Inputs of ``fit(rdd, sc)`` / ``predict(rdd, sc)`` and their placement.

The reference receives a PySpark RDD of ``(d,)`` float arrays built by
``sc.parallelize(X[, numSlices]).cache()`` (kmeans_spark.py:369, 418, 471,
518, 568).  This module accepts, duck-typed:

* ``LocalRDD`` — this package's stand-in for such an RDD
  (``LocalContext().parallelize(X, numSlices)`` mirrors ``sc.parallelize``),
* a real PySpark RDD (anything with ``mapPartitions`` / ``mapPartitionsWithIndex``),
* a NumPy array ``[n][d]`` (one partition),
* ``DeviceBlobs`` — a synthetic Gaussian-blob dataset generated directly in
  HBM (benchmarks; nothing on the host).

``place`` turns one into a ``Placement``: the global partition layout (needed
by the takeSample policy) and this rank's contiguous block of partitions and
rows.  With W ranks, rank r owns partitions ``[r*P//W, (r+1)*P//W)`` (a
one-partition input is cut into W row blocks), so concatenating the ranks'
predictions restores input order.

Ingestion is sharded at the source: the layout comes from a count pass
(for a PySpark RDD it runs on the executors: one ``(rows, width, dtype)``
triple per partition reaches the rank), and each rank then materialises only
its own partitions (``mapPartitionsWithIndex`` filtered to its block), so no
rank holds another rank's rows.  Rows needed by index later (takeSample
picks, kmeans_spark.py:72, 196) are gathered from the ranks' HBM
(``LloydRunner.rows``).

Rows are stored in HBM as float32 (the compute contract, see ``KMeans``): a
float64 input is rounded once at load, and every row the framework uses
afterwards -- assignment, sums, initial and replacement centroids -- is that
rounded row.
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass
from typing import Any, List, Optional, Sequence, Tuple

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

    def partition_len(self, i: int) -> int:
        return len(self._parts[i])

    def partition_array(self, i: int) -> Optional[np.ndarray]:
        """Partition i as a 2-D array (None when empty); only this rank's
        partitions are ever materialised (``place``)."""
        p = self._parts[i]
        if isinstance(p, np.ndarray) and p.ndim == 2:
            return p if len(p) else None
        items = list(p)
        return np.asarray(items) if items else None

    def partition_arrays(self) -> List[Optional[np.ndarray]]:
        return [self.partition_array(i) for i in range(len(self._parts))]

    def mapPartitionsWithIndex(self, f) -> "LocalRDD":
        return LocalRDD([list(f(i, iter(p))) for i, p in enumerate(self._parts)], self.ctx)

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
    local_rows: Optional[np.ndarray]  # this rank's rows (host, only its own), None for DeviceBlobs
    row0: int                        # global index of this rank's first row
    n_local: int
    n_global: int
    d: int
    dtype: Any
    blobs: Optional[DeviceBlobs] = None


def _count_width(it):
    """Per partition, on the executors: (rows, row width, dtype) -- no rows leave."""
    n, width, kind = 0, -1, ""
    for row in it:
        if n == 0:
            a = np.asarray(row)
            width, kind = int(a.size), a.dtype.str
        n += 1
    yield n, width, kind


def _layout(rdd) -> Tuple[List[int], Optional[int], Any]:
    """Global partition sizes, row width and dtype, without moving rows."""
    if isinstance(rdd, np.ndarray):
        if rdd.ndim != 2:
            raise ValueError("input array must be 2-D [n][d]")
        return [rdd.shape[0]], (rdd.shape[1] if rdd.shape[0] else None), rdd.dtype
    if isinstance(rdd, LocalRDD):
        sizes = [rdd.partition_len(i) for i in range(rdd.getNumPartitions())]
        for i, n in enumerate(sizes):
            if n:
                p = rdd._parts[i]
                first = np.asarray(p[0])
                return sizes, int(first.size), (p.dtype if isinstance(p, np.ndarray) else first.dtype)
        return sizes, None, np.float64
    if hasattr(rdd, "mapPartitions"):  # PySpark RDD (duck-typed)
        trip = rdd.mapPartitions(_count_width).collect()
        sizes = [int(t[0]) for t in trip]
        for n, width, kind in trip:
            if n:
                return sizes, int(width), np.dtype(kind)
        return sizes, None, np.float64
    raise TypeError(f"unsupported dataset type {type(rdd).__name__}: expected an RDD, LocalRDD, "
                    f"ndarray or DeviceBlobs")


def _own_rows(rdd, lo: int, hi: int, d: int, row_range: Optional[Tuple[int, int]] = None) -> np.ndarray:
    """This rank's rows: partitions [lo, hi), or rows [a, b) of the single
    partition 0 (row_range).  Only they are materialised / transferred."""
    if isinstance(rdd, np.ndarray):
        a, b = row_range if row_range else (0, rdd.shape[0])
        return rdd[a:b]
    if isinstance(rdd, LocalRDD):
        if row_range:
            p = rdd.partition_array(0)
            return p[row_range[0]:row_range[1]] if p is not None else np.zeros((0, d))
        mine = [rdd.partition_array(i) for i in range(lo, hi)]
        mine = [m.reshape(len(m), d) for m in mine if m is not None]
        return np.concatenate(mine) if mine else np.zeros((0, d))

    if row_range:
        a, b = row_range

        def keep(i, it):
            return itertools.islice(it, a, b) if i == 0 else iter(())
    else:
        def keep(i, it):
            return it if lo <= i < hi else iter(())
    rows = rdd.mapPartitionsWithIndex(keep).collect()
    return np.asarray(rows).reshape(len(rows), d) if rows else np.zeros((0, d))


def place(rdd, comm) -> Placement:
    if isinstance(rdd, DeviceBlobs):
        W, r = comm.world, comm.rank
        sizes = [((i + 1) * rdd.n) // W - (i * rdd.n) // W for i in range(W)]
        row0 = (r * rdd.n) // W
        P = max(1, int(rdd.partitions))
        layout = [((i + 1) * rdd.n) // P - (i * rdd.n) // P for i in range(P)]
        return Placement(global_sizes=layout, local_rows=None, row0=row0, n_local=sizes[r], n_global=rdd.n,
                         d=rdd.d, dtype=np.float64, blobs=rdd)
    sizes, d, dtype = _layout(rdd)
    if d is None:
        raise ValueError("Not enough data points (0) to initialize clusters")
    if not np.issubdtype(np.dtype(dtype), np.floating):
        dtype = np.float64
    W, r = comm.world, comm.rank
    if len(sizes) == 1 and W > 1:
        # one partition: cut into W row blocks (the takeSample layout is still ONE partition)
        n = sizes[0]
        a, b = (r * n) // W, ((r + 1) * n) // W
        local = _own_rows(rdd, 0, 1, d, row_range=(a, b))
        row0 = a
    else:
        P = len(sizes)
        lo, hi = (r * P) // W, ((r + 1) * P) // W
        local = _own_rows(rdd, lo, hi, d)
        row0 = int(sum(sizes[:lo]))
    if local.ndim != 2:
        local = local.reshape(len(local), d)
    return Placement(global_sizes=sizes, local_rows=local, row0=row0, n_local=len(local),
                     n_global=int(sum(sizes)), d=d, dtype=np.dtype(dtype))
