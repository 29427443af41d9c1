"""Run one attention shape `reps` times (for rocprofv3 --pmc passes)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from tools.attn_bench import SHAPES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="self4096")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    torch.manual_seed(0)
    for name, B, H, lq, lk, dh, bc in SHAPES:
        if name != args.shape:
            continue
        q = torch.randn(B * lq, H * dh, device="cuda").to(torch.bfloat16)
        kb = 1 if bc else B
        k = torch.randn(kb * lk, H * dh, device="cuda").to(torch.bfloat16)
        v = torch.randn(kb * lk, H * dh, device="cuda").to(torch.bfloat16)
        o = torch.empty_like(q)
        for _ in range(args.reps):
            ops.attention(q, k, v, o, batch=B, heads=H, lq=lq, lk=lk, dh=dh, scale=dh ** -0.5, kv_bcast=bc)
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
