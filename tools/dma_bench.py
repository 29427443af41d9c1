"""A/B of the LDS-DMA conv tiles (ids 20..26) against the register-staged tiles on the hot path's
conv shapes (bf16). Every tile must give bit-identical outputs (same k order, same MFMA)."""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

# name, B, H, W, c0, c1, cout, k, stride, up2, pad_tl (None = k//2)
SHAPES = [
    ("vae128@512", 16, 512, 512, 128, 0, 128, 3, 1, 0, None),
    ("vae128@1024", 8, 1024, 1024, 128, 0, 128, 3, 1, 0, None),
    ("vae256@256", 16, 256, 256, 256, 0, 256, 3, 1, 0, None),
    ("vae512@128", 16, 128, 128, 512, 0, 512, 3, 1, 0, None),
    ("vae512@64", 16, 64, 64, 512, 0, 512, 3, 1, 0, None),
    ("vae256to128@512", 16, 512, 512, 256, 0, 128, 3, 1, 0, None),
    ("vae_up512@64->128", 16, 64, 64, 512, 0, 512, 3, 1, 1, None),
    ("vae_up256@128->256", 16, 128, 128, 256, 0, 256, 3, 1, 1, None),
    ("vae_down128@512", 16, 512, 512, 128, 0, 128, 3, 2, 0, 0),
    ("unet320@64", 16, 64, 64, 320, 0, 320, 3, 1, 0, None),
    ("unet640@32", 16, 32, 32, 640, 0, 640, 3, 1, 0, None),
    ("unet1280to640@32", 16, 32, 32, 1280, 0, 640, 3, 1, 0, None),
    ("unet1920to640@32", 16, 32, 32, 1920, 0, 640, 3, 1, 0, None),
    ("unet960to640@32", 16, 32, 32, 960, 0, 640, 3, 1, 0, None),
    ("unet320to640@32", 16, 32, 32, 320, 0, 640, 3, 1, 0, None),
    ("unet640to1280@16", 16, 16, 16, 640, 0, 1280, 3, 1, 0, None),
    ("unet1280@16", 16, 16, 16, 1280, 0, 1280, 3, 1, 0, None),
    ("unet1280@8", 16, 8, 8, 1280, 0, 1280, 3, 1, 0, None),
    ("unet_cat640+320@64", 16, 64, 64, 640, 320, 320, 3, 1, 0, None),
    ("unet_cat1280+1280@8", 16, 8, 8, 1280, 1280, 1280, 3, 1, 0, None),
    ("unet_cat1280+1280@16", 16, 16, 16, 1280, 1280, 1280, 3, 1, 0, None),
    ("unet_cat1280+640@16", 16, 16, 16, 1280, 640, 1280, 3, 1, 0, None),
    ("unet640to320@64", 16, 64, 64, 640, 0, 320, 3, 1, 0, None),
    ("unet960to320@64", 16, 64, 64, 960, 0, 320, 3, 1, 0, None),
    ("lin1280x320", 1, 65536, 1, 1280, 0, 320, 1, 1, 0, None),
    ("lin320x960", 1, 65536, 1, 320, 0, 960, 1, 1, 0, None),
    ("lin320x2560", 1, 65536, 1, 320, 0, 2560, 1, 1, 0, None),
    ("lin320x320", 1, 65536, 1, 320, 0, 320, 1, 1, 0, None),
    ("lin1280x1280", 1, 4096, 1, 1280, 0, 1280, 1, 1, 0, None),
    ("lin640x640", 1, 16384, 1, 640, 0, 640, 1, 1, 0, None),
    ("lin1280x3840", 1, 4096, 1, 1280, 0, 3840, 1, 1, 0, None),
    ("lin5120x1280", 1, 4096, 1, 5120, 0, 1280, 1, 1, 0, None),
    ("lin2560x640", 1, 16384, 1, 2560, 0, 640, 1, 1, 0, None),
    ("tail3x20x20_128to192", 3, 20, 20, 128, 0, 192, 3, 1, 0, None),
    ("comp3x3_256to256@32", 16, 32, 32, 256, 0, 256, 3, 1, 0, None),
    ("comp5x5_256to128@32", 16, 32, 32, 256, 0, 128, 5, 1, 0, None),
    ("comp5x5_128to128@32", 16, 32, 32, 128, 0, 128, 5, 1, 0, None),
    ("comp3x3_256to384@32", 16, 32, 32, 256, 0, 384, 3, 1, 0, None),
    ("unet_cat640+320@32_1x1", 16, 32, 32, 640, 320, 640, 1, 1, 0, None),
    ("unet_cat1280+640@32_1x1", 16, 32, 32, 1280, 640, 640, 1, 1, 0, None),
]
TILES = (-1, 20, 21, 22, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38)


def bench(fn, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--only", default="")
    ap.add_argument("--tiles", default=",".join(str(t) for t in TILES))
    args = ap.parse_args()
    tiles = [int(t) for t in args.tiles.split(",")]
    torch.manual_seed(0)
    for name, B, H, W, c0, c1, cout, k, stride, up2, padtl in SHAPES:
        if args.only and not any(o in name for o in args.only.split(",")):
            continue
        x = torch.randn(B, H, W, c0, device="cuda").to(torch.bfloat16)
        x2 = torch.randn(B, H, W, c1, device="cuda").to(torch.bfloat16) if c1 else None
        cin = c0 + c1
        w = torch.randn(cout, cin, k, k, device="cuda") / math.sqrt(cin * k * k)
        p = ops.ConvParams.pack(w, torch.randn(cout, device="cuda"), stride=stride, pad=k // 2)
        hi, wi = (2 * H, 2 * W) if up2 else (H, W)
        kw = {}
        if padtl is not None:
            kw = dict(pad_t=padtl, pad_l=padtl, out_hw=((hi - k) // stride + 1, (wi - k) // stride + 1))
        ho, wo = kw.get("out_hw") or ((hi + 2 * (k // 2) - k) // stride + 1, (wi + 2 * (k // 2) - k) // stride + 1)
        res_t = torch.randn(B, ho, wo, cout, device="cuda").to(torch.bfloat16)
        flops = 2.0 * B * ho * wo * cout * cin * k * k
        outs, r = {}, dict(name=name)
        for t in tiles:
            ops.FORCE_TILE = t if t >= 0 else None
            ops.set_conv_option(5, 0 if t < 0 else 1)
            fn = lambda: ops.conv2d(x, p, x2=x2, up2=bool(up2), res=res_t, act=ops.SILU, **kw)  # noqa: E731
            outs[t] = fn()
            torch.cuda.synchronize()
            tm = min(bench(fn, args.reps) for _ in range(3))
            r[f"tf{t}"] = round(flops / tm / 1e12, 1)
        ref = outs[tiles[0]]
        r["identical"] = all(torch.equal(ref, o) for o in outs.values())
        if not r["identical"]:
            r["maxdiff"] = {t: (ref.float() - o.float()).abs().max().item() for t, o in outs.items()}
        print(json.dumps(r), flush=True)
    ops.set_conv_option(5, 1)
    ops.FORCE_TILE = None


if __name__ == "__main__":
    main()
