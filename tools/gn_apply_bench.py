"""GroupNorm apply (rdeic_groupnorm_apply, the materialised UNet / control-net path) on the bench's shapes:
us per launch and GB/s (read + write of the bf16 activations), min over 3 runs of 20 launches.
usage (GPU box): python tools/gn_apply_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

SHAPES = [(16, 64, 64, 320), (16, 64, 64, 640), (16, 64, 64, 960), (16, 32, 32, 640), (16, 32, 32, 1280),
          (16, 32, 32, 1920), (16, 16, 16, 1280), (16, 16, 16, 2560), (16, 8, 8, 1280), (16, 8, 8, 2560)]


def main():
    torch.manual_seed(0)
    for n, h, w, c in SHAPES:
        x = torch.randn(n, h, w, c, device="cuda").to(torch.bfloat16)
        ab = torch.randn(n, c, 2, device="cuda")
        y = torch.empty_like(x)
        ops.group_norm_apply(x, ab, True, out=y)
        best = 1e9
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                ops.group_norm_apply(x, ab, True, out=y)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
        gb = 2 * x.numel() * 2 / 1e9
        print(json.dumps({"shape": [n, h, w, c], "us": round(best, 2), "gbs": round(gb / (best * 1e-6), 1)}), flush=True)


if __name__ == "__main__":
    main()
