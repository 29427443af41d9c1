"""Host rANS encode throughput (diagnostics): ns/symbol of the tabled encoder on one thread and
the batch over T threads, on bench-like symbol statistics (~0.08 bpp: almost every symbol the
most probable value of a low-scale row)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import coders  # noqa: E402

t = coders.GaussianTables()
rng = np.random.default_rng(0)
n = 262144
idx = np.where(rng.random((16, n)) < 0.9, 0, rng.integers(0, 12, size=(16, n))).astype(np.int32)
sym = np.where(rng.random((16, n)) < 0.003, rng.integers(-2, 3, size=(16, n)), 0).astype(np.int32)
for th in (1, 2, 4, 8, 16):
    cnt = th if th > 1 else 1
    s, i = sym[:cnt], idx[:cnt]
    coders.rans_encode_batch(s, i, t, threads=th)
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        out = coders.rans_encode_batch(s, i, t, threads=th)
    dt = (time.perf_counter() - t0) / reps
    print(f"threads {th:2d} images {cnt:2d}: {dt * 1e3:7.2f} ms  ({dt / n * 1e9:6.2f} ns/sym per thread-image), "
          f"{np.mean([len(o) for o in out]):.0f} B/image", flush=True)
