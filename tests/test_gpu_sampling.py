"""takeSample's Bernoulli pass on the GPU (km_bernoulli_sample, csrc/km_sample.hip)
against the host restatement (sampling.py, itself pinned to the reference's
takeSample under the PySpark stand-in by tests/test_host.py): identical picks,
for seeds above 2^32, odd warm-up word counts, partitions that end inside a
twist block, empty and one-row partitions (kmeans_spark.py:72, :196)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    import kmeans_amd as ka
    from kmeans_amd.engine import HipEngine
    return HipEngine(0)


@pytest.mark.parametrize("sizes,fraction,seed", [
    ([1000, 313, 1, 0, 70001], 0.01, 42),
    ([400_000] * 4, 3e-5, 1_700_000_123),
    ([624, 623, 625, 311, 312], 0.5, 2 ** 40 + 7),
    ([100_000, 250_000], 0.001, 9_223_372_036_854_775_807),
    ([5_000_000], 2e-6, 6),
])
def test_device_bernoulli_equals_host(engine, sizes, fraction, seed):
    from kmeans_amd import sampling
    bases = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    mine = [p for p in range(len(sizes)) if sizes[p] > 0]
    want = np.concatenate([sampling._partition_picks(p, int(bases[p]), sizes[p], fraction, seed) for p in mine])
    got = engine.bernoulli(np.array([seed ^ p for p in mine], dtype=np.uint64),
                           np.array([sizes[p] for p in mine]), bases[mine], fraction)
    assert got is not None
    np.testing.assert_array_equal(got, want)


def test_device_bernoulli_equals_cpython_literals(engine):
    # the literal picks of CPython's random module (tests/test_host.py
    # CPYTHON_PICKS): the device MT19937 against CPython itself, not only
    # against the host restatement
    from test_host import CPYTHON_PICKS
    for sizes, fraction, seed, want in CPYTHON_PICKS:
        bases = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
        mine = [p for p in range(len(sizes)) if sizes[p] > 0]
        got = engine.bernoulli(np.array([seed ^ p for p in mine], dtype=np.uint64),
                               np.array([sizes[p] for p in mine]), bases[mine], fraction)
        assert got is not None
        assert got.tolist() == want


def test_take_sample_with_device_pass(engine):
    from kmeans_amd import sampling
    sizes = [300_000, 200_001, 0, 150_000]
    for num, seed in [(7, 42), (256, 1_699_999_999), (1, 3), (5, -987654321), (9, -(2 ** 63)), (4, 2 ** 64 + 5)]:
        assert sampling.take_sample(sizes, num, seed, device=engine.bernoulli) == \
            sampling.take_sample(sizes, num, seed)


def test_device_pass_overflow_falls_back(engine):
    # more picks than the device slots (4x expectation + 64) -> None, host path
    from kmeans_amd import sampling
    got = engine.bernoulli(np.array([5], dtype=np.uint64), np.array([100_000]), np.array([0]), 0.0)
    assert got is not None and len(got) == 0
    sizes = [100_000, 100_000]
    assert sampling.take_sample(sizes, 3, 11, device=lambda *a: None) == sampling.take_sample(sizes, 3, 11)
