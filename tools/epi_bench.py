"""Epilogue cost of the LDS-DMA conv tiles: the same conv timed with a plain store, with a residual
add, with the fused GroupNorm statistics and with both (HIP events over repeated launches).
usage: python tools/epi_bench.py [--tiles 34,35,32] [--only vae128]"""
import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

# name, B, H, W, cin, cout, k
SHAPES = [
    ("vae128@512", 16, 512, 512, 128, 128, 3),
    ("vae256@256", 16, 256, 256, 256, 256, 3),
    ("vae512@128", 16, 128, 128, 512, 512, 3),
    ("vae256to128@512", 16, 512, 512, 256, 128, 3),
    ("lin128@512", 16, 512, 512, 128, 128, 1),
    ("unet320@64", 16, 64, 64, 320, 320, 3),
    ("unet640@32", 16, 32, 32, 640, 640, 3),
    ("lin320x320", 16, 64, 64, 320, 320, 1),
    ("lin640x640", 16, 32, 32, 640, 640, 1),
    ("lin1280x1280", 16, 16, 16, 1280, 1280, 1),
]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="34,35,32")
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=10)
    args = ap.parse_args()
    torch.manual_seed(0)
    for name, B, H, W, cin, cout, k in SHAPES:
        if args.only and args.only not in name:
            continue
        x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device="cuda") / math.sqrt(cin * k * k)
        p = ops.ConvParams.pack(w, torch.randn(cout, device="cuda"), stride=1, pad=k // 2)
        res = torch.randn(B, H, W, cout, device="cuda").to(torch.bfloat16)
        flops = 2.0 * B * H * W * cout * cin * k * k
        row = {"name": name}
        for t in [int(s) for s in args.tiles.split(",")]:
            ops.FORCE_TILE = t
            for var, kw in (("plain", {}), ("res", {"res": res}), ("stats", {"stats": True}),
                            ("res+stats", {"res": res, "stats": True})):
                ms = timeit(lambda: ops.conv2d(x, p, **kw), args.reps)
                row[f"{t}:{var}"] = round(flops / ms / 1e9, 1)
        ops.FORCE_TILE = None
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
