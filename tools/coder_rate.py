"""Host rANS coder throughput per thread (the coder-thread budget of 8 ranks on one host).

Encodes and decodes a batch of config-2-shaped streams (262,144 symbols per 512^2 image) through the library's
own entry points (rdeic_rans_encode_batch_t / rdeic_rans_decode_batch) with 1 and with N threads, and prints
symbols/s per thread and the threads one GPU's codec rate needs. Symbols follow the Gaussian-conditional model at
scale indexes drawn like the bench's ~0.08 bpp streams (mostly the smallest scales).
usage: python tools/coder_rate.py [IMAGES] [THREADS] [IMG_PER_S]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import coders  # noqa: E402


def main():
    images = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    nthreads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    img_per_s = float(sys.argv[3]) if len(sys.argv) > 3 else 150.0
    n = 262144
    t = coders.GaussianTables()
    rng = np.random.default_rng(231)
    # scale indexes: geometric over the 64 levels (low bpp: small scales dominate); symbols ~ N(0, scale)
    idx = np.minimum(rng.geometric(0.35, size=(images, n)) - 1, 63).astype(np.int32)
    scales = t.scale_table.numpy()[idx]
    sym = np.rint(rng.standard_normal((images, n)) * scales).astype(np.int32)
    out = {"images": images, "symbols_per_image": n}
    for th in (1, nthreads):
        coders.rans_encode_batch(sym[:2], idx[:2], t, threads=th)  # warm (tables, pools)
        t0 = time.perf_counter()
        bodies = coders.rans_encode_batch(sym, idx, t, threads=th)
        te = time.perf_counter() - t0
        decs = [coders.RansDecoder(b) for b in bodies]
        t0 = time.perf_counter()
        got = coders.rans_decode_batch(decs, idx, t, threads=th)
        td = time.perf_counter() - t0
        assert np.array_equal(got, sym), "round trip"
        out[f"threads_{th}"] = {"encode_msym_s": round(images * n / te / 1e6, 2),
                                "decode_msym_s": round(images * n / td / 1e6, 2),
                                "bytes_per_image": int(np.mean([len(b) for b in bodies]))}
    one = out["threads_1"]
    need = img_per_s * n / 1e6  # Msym/s each way per GPU
    out["per_gpu_msym_s_each_way"] = round(need, 2)
    out["threads_per_gpu_needed"] = round(need / one["encode_msym_s"] + need / one["decode_msym_s"], 2)
    out["threads_per_node_8_gpus"] = round(8 * out["threads_per_gpu_needed"], 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
