"""Time takeSample's Bernoulli pass for the c3 layout (100M rows, 256
partitions): GPU pass vs the host threads (GPU box)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import kmeans_amd as ka
from kmeans_amd import sampling
from kmeans_amd.engine import HipEngine
eng = HipEngine(0)
n, P = 100_000_000, 256
sizes = [((i + 1) * n) // P - (i * n) // P for i in range(P)]
for num in (1, 10):
    t0 = time.perf_counter(); a = sampling.take_sample(sizes, num, 1_700_000_000 + num, device=eng.bernoulli)
    t1 = time.perf_counter(); b = sampling.take_sample(sizes, num, 1_700_000_000 + num)
    t2 = time.perf_counter()
    print(f"num={num}: device {1e3*(t1-t0):.1f} ms, host {1e3*(t2-t1):.1f} ms, equal={a == b}")
