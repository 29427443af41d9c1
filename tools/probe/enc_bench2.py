"""Encoder batch scaling on the box: per-image cost with many images per thread (steady state) vs
one image per thread (pool wake-up latency included)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import coders  # noqa: E402

t = coders.GaussianTables()
rng = np.random.default_rng(0)
n = 262144
N = 64
idx = np.where(rng.random((N, n)) < 0.9, 0, rng.integers(0, 12, size=(N, n))).astype(np.int32)
sym = np.where(rng.random((N, n)) < 0.003, rng.integers(-2, 3, size=(N, n)), 0).astype(np.int32)
for th, cnt in ((4, 16), (8, 16), (16, 16), (16, 64), (4, 64), (8, 64)):
    s, i = sym[:cnt], idx[:cnt]
    coders.rans_encode_batch(s, i, t, threads=th)
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        coders.rans_encode_batch(s, i, t, threads=th)
    dt = (time.perf_counter() - t0) / reps
    print(f"threads {th:2d} images {cnt:2d}: {dt * 1e3:7.2f} ms ({dt * th / cnt * 1e3:5.2f} ms per image-thread)",
          flush=True)
print("cpus", os.sched_getaffinity(0).__len__(), flush=True)
