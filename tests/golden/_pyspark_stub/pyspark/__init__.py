"""In-memory stand-in for the slice of the PySpark RDD API that
``/root/reference/kmeans_spark.py`` touches.

TEST INFRASTRUCTURE ONLY.  It lets ``tests/golden/make_golden.py`` import the
reference module unmodified in this container (pyspark / a JVM are absent) so
that golden input/output vectors can be generated from the reference's own
``KMeans``.  Nothing here ships; nothing here is copied from PySpark.

Semantics mirrored from PySpark 3.x where the reference depends on them:
  * ``parallelize(X, numSlices)`` cuts the sequence into contiguous slices
    ``[i*n//s, (i+1)*n//s)`` (PySpark ``SparkContext.parallelize``).
  * ``reduceByKey`` does a map-side left fold per partition (createCombiner =
    identity, mergeValue = f), then merges the per-partition combiners in
    partition order.  The sum order is therefore deterministic here (it is not
    in real Spark).
  * ``sum`` folds per-partition sums in partition order, starting from 0.
  * ``takeSample(False, num, seed)`` follows PySpark's algorithm
    (count -> fraction -> per-partition Bernoulli sampler seeded with
    ``seed ^ split`` -> retry -> ``Random(seed).shuffle`` -> truncate); the
    same index-level restatement lives in the product
    (``..._amd/sampling.py``) and in ``oracle/kmeans_oracle.py``.
"""
import math
import random
import sys

__all__ = ["SparkContext", "RDD", "Broadcast"]


class Broadcast:
    def __init__(self, value):
        self.value = value

    def unpersist(self, blocking=False):
        pass


def _fraction_for_sample_size(num, total):
    # PySpark RDD._computeFractionForSampleSize, without replacement
    fraction = float(num) / total
    delta = 0.00005
    gamma = -math.log(delta) / total
    return min(1.0, fraction + gamma + math.sqrt(gamma * gamma + 2 * gamma * fraction))


class RDD:
    def __init__(self, partitions, ctx):
        self._parts = [list(p) for p in partitions]
        self.ctx = ctx

    # -- persistence (no-ops) -------------------------------------------
    def cache(self):
        return self

    def unpersist(self, blocking=False):
        return self

    def getNumPartitions(self):
        return len(self._parts)

    # -- transformations (eager) -----------------------------------------
    def mapPartitions(self, f):
        return RDD([list(f(iter(p))) for p in self._parts], self.ctx)

    def repartition(self, n):
        flat = [x for p in self._parts for x in p]
        return self.ctx.parallelize(flat, n)

    def reduceByKey(self, f):
        combined = []
        for p in self._parts:
            d = {}
            for key, val in p:
                d[key] = f(d[key], val) if key in d else val
            combined.append(d)
        out = {}
        for d in combined:
            for key, val in d.items():
                out[key] = f(out[key], val) if key in out else val
        return RDD([list(out.items())], self.ctx)

    # -- actions -----------------------------------------------------------
    def collect(self):
        return [x for p in self._parts for x in p]

    def count(self):
        return sum(len(p) for p in self._parts)

    def sum(self):
        total = 0
        for p in self._parts:
            s = 0
            for x in p:
                s = s + x
            total = total + s
        return total

    def _sample_pass(self, fraction, seed):
        out = []
        for split, p in enumerate(self._parts):
            rng = random.Random(seed ^ split)
            for _ in range(10):
                rng.randint(0, 1)
            for obj in p:
                if rng.random() < fraction:
                    out.append(obj)
        return out

    def takeSample(self, withReplacement, num, seed=None):
        if withReplacement:
            raise NotImplementedError("stub: only withReplacement=False is used")
        if num < 0:
            raise ValueError("Sample size cannot be negative.")
        if num == 0:
            return []
        total = self.count()
        if total == 0:
            return []
        if seed is None:
            seed = random.randint(0, sys.maxsize)
        rand = random.Random(seed)
        if num >= total:
            samples = self.collect()
            rand.shuffle(samples)
            return samples
        fraction = _fraction_for_sample_size(num, total)
        samples = self._sample_pass(fraction, seed)
        while len(samples) < num:
            seed = rand.randint(0, sys.maxsize)
            samples = self._sample_pass(fraction, seed)
        rand.shuffle(samples)
        return samples[0:num]


class SparkContext:
    def __init__(self, master=None, appName=None, defaultParallelism=4, **kw):
        self.defaultParallelism = defaultParallelism

    def parallelize(self, c, numSlices=None, numPartitions=None):
        n_slices = numSlices or numPartitions or self.defaultParallelism
        data = list(c)
        n = len(data)
        parts = [data[(i * n) // n_slices:((i + 1) * n) // n_slices] for i in range(n_slices)]
        return RDD(parts, self)

    def broadcast(self, value):
        return Broadcast(value)

    def setLogLevel(self, level):
        pass

    def stop(self):
        pass
