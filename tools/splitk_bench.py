"""Split-K A/B on the UNet's small-grid 3x3 layers (bf16, B=16): the table's tile without split
against forced k-split counts (split-K runs on the heuristic DMA tile, fixed-order reduce)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

SHAPES = [("unet640@32", 16, 32, 32, 640, 640, (2, 3, 4, 6)), ("unet1280@16", 16, 16, 16, 1280, 1280, (2, 3)),
          ("unet1280@8", 16, 8, 8, 1280, 1280, (3, 4, 5, 6, 7, 8)), ("unet2560@8", 16, 8, 8, 2560, 1280, (4, 6, 7, 8)),
          # the entropy model's nets at y = 32x32 (512^2 images): 5x5 context / parameter convs, 3x3 g_s
          ("ep5x5 256->128@32", 16, 32, 32, 256, 128, (2, 3, 4, 6), 5), ("ep5x5 192->256@32", 16, 32, 32, 192, 256, (2, 3, 4), 5),
          ("gs3x3 256->256@32", 16, 32, 32, 256, 256, (2, 3, 4)), ("c3x3 256->256@16", 16, 16, 16, 256, 256, (2, 3, 4, 6, 9)),
          # control net (0.2 x the UNet widths) at its 8x8 level: 16 tiles of 128x128 at B=16
          ("c3x3 256->256@8", 16, 8, 8, 256, 256, (2, 3, 4, 6, 9, 12))]


def timeit(fn, reps=10):
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
    orig = ops._splitk_count
    only = sys.argv[1:]
    for name, B, H, W, cin, cout, splits, *kk in SHAPES:
        if only and not any(o in name for o in only):
            continue
        k = kk[0] if kk else 3
        x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device="cuda") / math.sqrt(cin * k * k)
        p = ops.ConvParams.pack(w, torch.randn(cout, device="cuda"), stride=1, pad=k // 2)
        emb = torch.randn(B, cout, device="cuda") if name.startswith("unet") else None
        flops = 2.0 * B * H * W * cout * cin * k * k
        row = {"name": name}
        key = ops.tile_key(B * H * W, cin, 0, p, False, 0, False, emb is not None, 0, torch.bfloat16)
        row["table_tile"] = ops.TILE_TABLE.get(key)
        for sp in (1,) + tuple(splits):
            ops._splitk_count = (lambda *a, _s=sp, **k: _s)
            try:
                fn = lambda: ops.conv2d(x, p, emb=emb)  # noqa: E731
                ms = timeit(fn)
            finally:
                ops._splitk_count = orig
            row[f"s{sp}"] = round(flops / ms / 1e9, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
