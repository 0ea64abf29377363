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
by the takeSample policy) and this rank's contiguous block of rows.  With N
rows over W ranks, rank r owns global rows ``[r*N//W, (r+1)*N//W)`` whatever
the partition boundaries (the reference's own inputs have 1-4 partitions,
kmeans_spark.py:418, 561-568, so whole partitions per rank would leave GPUs
idle); a rank's block may start and end inside partitions.  The takeSample
layout stays the dataset's own partitioning, so the sampled rows and the whole
run are the same for any W; concatenating the ranks' predictions restores
input order.

Ingestion is sharded at the source: the layout comes from a count pass
(for a PySpark RDD it runs on the executors: one ``(rows, width, dtype)``
triple per partition reaches the rank), and each rank then materialises only
its own rows (``mapPartitionsWithIndex`` slicing each overlapping partition to
the rank's row range), so no rank holds another rank's rows.  Rows needed by index later (takeSample
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


def _segments(sizes: Sequence[int], a: int, b: int) -> List[Tuple[int, int, int]]:
    """Global rows [a, b) as (partition, first, stop) pieces, in row order."""
    out, start = [], 0
    for i, n in enumerate(sizes):
        lo, hi = max(a, start), min(b, start + n)
        if lo < hi:
            out.append((i, lo - start, hi - start))
        start += n
    return out


def _own_rows(rdd, segs: List[Tuple[int, int, int]], d: int) -> np.ndarray:
    """This rank's rows: the given partition pieces.  Only they are
    materialised / transferred."""
    if isinstance(rdd, np.ndarray):
        return np.concatenate([rdd[lo:hi] for _, lo, hi in segs]) if segs else np.zeros((0, d))
    if isinstance(rdd, LocalRDD):
        mine = []
        for i, lo, hi in segs:
            p = rdd.partition_array(i)
            if p is not None:
                mine.append(p[lo:hi].reshape(hi - lo, d))
        return np.concatenate(mine) if mine else np.zeros((0, d))
    want = {i: (lo, hi) for i, lo, hi in segs}

    def keep(i, it):
        if i not in want:
            return iter(())
        lo, hi = want[i]
        return itertools.islice(it, lo, hi)
    rows = rdd.mapPartitionsWithIndex(keep).collect()  # partitions come back in index order
    return np.asarray(rows).reshape(len(rows), d) if rows else np.zeros((0, d))


def rank_rows(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Global row range [a, b) of a rank: balanced to one row."""
    return (rank * n) // world, ((rank + 1) * n) // world


class EmptyDataset(ValueError):
    """The dataset has no rows.  ``fit`` turns it into the reference's init
    error (takeSample returns [] for an empty RDD, kmeans_spark.py:72-74);
    ``predict`` returns an empty result (its lazy map over no rows)."""


def place(rdd, comm) -> Placement:
    if isinstance(rdd, DeviceBlobs):
        a, b = rank_rows(rdd.n, comm.world, comm.rank)
        P = max(1, int(rdd.partitions))
        layout = [((i + 1) * rdd.n) // P - (i * rdd.n) // P for i in range(P)]
        return Placement(global_sizes=layout, local_rows=None, row0=a, n_local=b - a, n_global=rdd.n,
                         d=rdd.d, dtype=np.float64, blobs=rdd)
    sizes, d, dtype = _layout(rdd)
    if d is None:
        raise EmptyDataset("the dataset has no rows")
    if not np.issubdtype(np.dtype(dtype), np.floating):
        dtype = np.float64
    # balanced row blocks across partition boundaries (the takeSample layout
    # stays the dataset's partitions)
    a, b = rank_rows(int(sum(sizes)), comm.world, comm.rank)
    local = _own_rows(rdd, _segments(sizes, a, b), d)
    row0 = a
    if local.ndim != 2:
        local = local.reshape(len(local), d)
    return Placement(global_sizes=sizes, local_rows=local, row0=row0, n_local=len(local),
                     n_global=int(sum(sizes)), d=d, dtype=np.dtype(dtype))
