"""Run one conv shape `reps` times on one path (for rocprofv3 --pmc passes)."""
import argparse
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from tools.conv_bench import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="vae128@512")
    ap.add_argument("--paths", default="2,3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tile", type=int, default=None, help="force this tile id (ops.FORCE_TILE)")
    args = ap.parse_args()
    torch.manual_seed(0)
    for name, B, H, W, cin, cout, k, stride in SHAPES:
        if name != args.shape:
            continue
        x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device="cuda") / math.sqrt(cin * k * k)
        p = ops.ConvParams.pack(w, torch.randn(cout, device="cuda"), stride=stride, pad=k // 2)
        ops.FORCE_TILE = args.tile
        for path in [int(v) for v in args.paths.split(",")]:
            ops.set_conv_path(path)
            for _ in range(args.reps):
                ops.conv2d(x, p)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
