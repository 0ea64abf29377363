"""Row sampling policy of the reference: ``rdd.takeSample(False, num, seed)``.

Used for the initial centroids (kmeans_spark.py:72, ``seed=self.seed``) and for
empty-cluster replacement (kmeans_spark.py:196, ``seed=int(time.time())``).
Sampling without replacement never looks at row values, so it is restated at
index level over the dataset's partition layout; the caller then fetches the
selected rows.  Algorithm: PySpark 3.x ``RDD.takeSample`` +
``RDDSampler`` (fraction from ``_computeFractionForSampleSize``, Bernoulli
sampler per partition seeded ``seed ^ split`` with 10 warm-up draws, retry
with a fresh seed until enough rows, ``Random(seed).shuffle``, truncate).
PySpark is not installed here, so agreement with a real Spark run is
unpinned; agreement with the reference under the test stand-in is checked by
``tests/test_host.py``.
"""
from __future__ import annotations

import math
import random
import sys
from typing import List, Optional, Sequence

import numpy as np


def _fraction(num: int, total: int) -> float:
    fraction = float(num) / total
    delta = 0.00005
    gamma = -math.log(delta) / total
    return min(1.0, fraction + gamma + math.sqrt(gamma * gamma + 2 * gamma * fraction))


def _mt_init_by_array(key: List[int]) -> np.ndarray:
    """MT19937 ``init_by_array`` (the seeding CPython's ``random.seed(int)`` uses)."""
    mt = [0] * 624
    mt[0] = 19650218
    for i in range(1, 624):
        mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
    i, j, kl = 1, 0, len(key)
    for _ in range(max(624, kl)):
        mt[i] = ((mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525)) + key[j] + j) & 0xFFFFFFFF
        i += 1
        j += 1
        if i >= 624:
            mt[0] = mt[623]
            i = 1
        if j >= kl:
            j = 0
    for _ in range(623):
        mt[i] = ((mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941)) - i) & 0xFFFFFFFF
        i += 1
        if i >= 624:
            mt[0] = mt[623]
            i = 1
    mt[0] = 0x80000000
    return np.array(mt, dtype=np.uint32)


def _python_random_stream(seed: int) -> np.random.RandomState:
    """A NumPy MT19937 positioned exactly where ``r = random.Random(seed)`` is
    after RDDSampler's ``for _ in range(10): r.randint(0, 1)``; its
    ``random_sample()`` then yields the same doubles as ``r.random()``
    (same generator, same 53-bit construction; checked in tests)."""
    a = abs(int(seed))
    key = []
    while True:
        key.append(a & 0xFFFFFFFF)
        a >>= 32
        if a == 0:
            break
    rs = np.random.RandomState()
    rs.set_state(("MT19937", _mt_init_by_array(key), 624, 0, 0.0))
    accepted = 0
    while accepted < 10:  # randint(0,1) = getrandbits(2) with rejection of values >= 2
        w = int(rs.randint(0, 2 ** 32, size=1, dtype=np.uint32)[0])
        if (w >> 30) < 2:
            accepted += 1
    return rs


def _bernoulli_pass_py(partition_sizes: Sequence[int], fraction: float, seed: int) -> List[int]:
    picked: List[int] = []
    base = 0
    for split, size in enumerate(partition_sizes):
        rng = random.Random(seed ^ split)
        for _ in range(10):  # RDDSampler mixes the close per-split seeds
            rng.randint(0, 1)
        draw = rng.random
        picked.extend(base + i for i in range(size) if draw() < fraction)
        base += size
    return picked


def _partition_picks(split: int, base: int, size: int, fraction: float, seed: int) -> np.ndarray:
    """Global indices of one partition's Bernoulli sample (its own stream)."""
    rs = _python_random_stream(seed ^ split)
    chunk = 1 << 24
    out = []
    for s in range(0, size, chunk):
        u = rs.random_sample(min(chunk, size - s))   # releases the GIL: partitions run in parallel threads
        out.append(np.nonzero(u < fraction)[0] + (base + s))
    return np.concatenate(out) if out else np.zeros(0, dtype=np.int64)


def _bernoulli_pass(partition_sizes: Sequence[int], fraction: float, seed: int, comm=None,
                    device=None) -> List[int]:
    """Every partition's picks in partition order.  The partitions are
    independent streams (seed ^ split): they are split over the ranks of
    ``comm`` (partition p on rank p % world, results all-gathered), and run
    on this rank's GPU (``device`` = HipEngine.bernoulli, one wave per
    partition) or else over host threads; the result does not depend on
    any of that."""
    if sum(partition_sizes) <= 65536:
        return _bernoulli_pass_py(partition_sizes, fraction, seed)
    bases = np.concatenate([[0], np.cumsum(partition_sizes)[:-1]]).astype(np.int64)
    world = comm.world if comm is not None else 1
    rank = comm.rank if comm is not None else 0
    mine = [p for p in range(len(partition_sizes)) if p % world == rank and partition_sizes[p] > 0]
    parts = None
    # the streams' MT keys: random.Random(seed ^ p) seeds with abs(seed ^ p)
    # (negative seeds are valid); the device pass takes 64-bit keys, larger
    # ones stay on the host path
    keys = [abs(int(seed) ^ p) for p in mine]
    if device is not None and mine and max(keys) < 2 ** 64:
        picks = device(np.array(keys, dtype=np.uint64),
                       np.array([partition_sizes[p] for p in mine], dtype=np.int64), bases[mine], fraction)
        parts = None if picks is None else [picks]
    if parts is None and len(mine) > 1:
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=min(len(mine), 16)) as ex:
            parts = list(ex.map(lambda p: _partition_picks(p, int(bases[p]), int(partition_sizes[p]), fraction,
                                                           seed), mine))
    elif parts is None:
        parts = [_partition_picks(p, int(bases[p]), int(partition_sizes[p]), fraction, seed) for p in mine]
    local = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int64)
    if world > 1:
        local = np.concatenate(comm.allgather_array(local.astype(np.int64)))
    return np.sort(local, kind="stable").tolist()


def take_sample(partition_sizes: Sequence[int], num: int, seed: Optional[int], comm=None,
                device=None) -> List[int]:
    """Global row indices that ``takeSample(False, num, seed)`` returns, in order.
    With ``comm`` every rank must call it with the same arguments; ``device``
    runs the Bernoulli passes on the GPU (see ``_bernoulli_pass``)."""
    if num < 0:
        raise ValueError("Sample size cannot be negative.")
    total = int(sum(partition_sizes))
    if num == 0 or total == 0:
        return []
    if seed is None:
        seed = random.randint(0, sys.maxsize)
        if comm is not None and comm.world > 1:
            seed = comm.broadcast_obj(seed)
    rand = random.Random(seed)
    if num >= total:
        idx = list(range(total))
        rand.shuffle(idx)
        return idx
    fraction = _fraction(num, total)
    samples = _bernoulli_pass(partition_sizes, fraction, seed, comm, device)
    while len(samples) < num:
        seed = rand.randint(0, sys.maxsize)
        samples = _bernoulli_pass(partition_sizes, fraction, seed, comm, device)
    rand.shuffle(samples)
    return samples[0:num]
