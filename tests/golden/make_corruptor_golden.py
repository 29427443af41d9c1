"""Golden vectors for the robustness corruptors, from the reference's own experiments/corruptors.py
run in this container. Output: tests/golden/corruptors.npz (inputs + corrupted outputs).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_corruptor_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

BYTE_CASES = [("random", 0.001, 42), ("random", 0.01, 7), ("random", 0.05, 3), ("burst", 0.001, 42),
              ("burst", 0.01, 7), ("burst", 0.05, 3), ("random", 0.0, 1), ("burst", 0.00001, 5)]
LATENT_CASES = [("mask_replace", 0.05, 42), ("mask_replace", 0.3, 9), ("additive", 0.1, 42), ("additive", 1.0, 4)]


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    from experiments import corruptors as C
    rng = np.random.RandomState(1234)
    data = rng.randint(0, 256, size=2600).astype(np.uint8).tobytes()
    out = {"data": np.frombuffer(data, dtype=np.uint8)}
    for k, (kind, rate, seed) in enumerate(BYTE_CASES):
        f = C.bit_flip_bytes(data, rate, seed) if kind == "random" else C.burst_flip_bytes(data, rate, 8.0, seed)
        out[f"bytes{k}_kind"] = np.frombuffer(kind.encode(), dtype=np.uint8)
        out[f"bytes{k}_rate"] = np.float64(rate)
        out[f"bytes{k}_seed"] = np.int64(seed)
        out[f"bytes{k}_out"] = np.frombuffer(f, dtype=np.uint8)
    lat = torch.randn((1, 4, 16, 16), generator=torch.Generator().manual_seed(5)) * 1.5
    out["latent"] = lat.numpy()
    lo, hi = C.estimate_latent_range(lat)
    out["latent_range"] = np.array([lo, hi])
    for k, (mode, rate, seed) in enumerate(LATENT_CASES):
        r = C.latent_corrupt(lat, mode, rate, seed, (lo, hi))
        out[f"lat{k}_mode"] = np.frombuffer(mode.encode(), dtype=np.uint8)
        out[f"lat{k}_rate"] = np.float64(rate)
        out[f"lat{k}_seed"] = np.int64(seed)
        out[f"lat{k}_out"] = r.numpy()
    path = os.path.join(HERE, "corruptors.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
