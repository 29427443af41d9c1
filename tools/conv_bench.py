"""Conv kernel micro-benchmark on the hot path's conv shapes (bf16, batch 16 @ 512x512 images).
Interleaves conv paths / options in one process and checks that all produce bit-identical
outputs (same k-order, same MFMA)."""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

SHAPES = [  # (name, B, H, W, cin, cout, k, stride)
    ("unet320@64", 16, 64, 64, 320, 320, 3, 1),
    ("unet640@32", 16, 32, 32, 640, 640, 3, 1),
    ("unet1280@16", 16, 16, 16, 1280, 1280, 3, 1),
    ("unet1280@8", 16, 8, 8, 1280, 1280, 3, 1),
    ("unet_cat2560@8", 16, 8, 8, 2560, 1280, 3, 1),
    ("vae128@512", 16, 512, 512, 128, 128, 3, 1),
    ("vae256@256", 16, 256, 256, 256, 256, 3, 1),
    ("vae512@128", 16, 128, 128, 512, 512, 3, 1),
    ("vae512@64", 16, 64, 64, 512, 512, 3, 1),
    ("linear320x1280 (ff)", 16, 64, 64, 320, 2560, 1, 1),
    ("linear320x320", 16, 64, 64, 320, 320, 1, 1),
    ("vae256to128@512", 16, 512, 512, 256, 128, 3, 1),
]


def bench(fn, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--paths", default="0,2")
    ap.add_argument("--epi", default="1", help="comma list of epilogue modes to A/B (1 vector, 0 scalar)")
    ap.add_argument("--pf2", default="0", help="comma list of register-prefetch modes to A/B (1 two-deep, 0 one)")
    ap.add_argument("--swz", default="1", help="comma list of LDS layouts to A/B (1 swizzled, 0 padded)")
    ap.add_argument("--splitk", default="0", help="comma list: 1 = allow split-K (UNet mode)")
    ap.add_argument("--tiles", default="-1", help="comma list of forced tile candidates (-1 auto, 0..5)")
    args = ap.parse_args()
    torch.manual_seed(0)
    res = []
    for name, B, H, W, cin, cout, k, stride in SHAPES:
        if args.only and args.only not in name:
            continue
        x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
        w = torch.randn(cout, cin, k, k, device="cuda") / math.sqrt(cin * k * k)
        p = ops.ConvParams.pack(w, torch.randn(cout, device="cuda"), stride=stride, pad=k // 2)
        res_t = torch.randn(B, H // stride, W // stride, cout, device="cuda").to(torch.bfloat16)
        paths = [(int(v), int(e), int(f), int(z), int(k), int(t)) for v in args.paths.split(",")
                 for e in args.epi.split(",") for f in args.pf2.split(",") for z in args.swz.split(",")
                 for k in args.splitk.split(",") for t in args.tiles.split(",")]
        outs = {}
        times = {q: [] for q in paths}
        fn = lambda: ops.conv2d(x, p, res=res_t, act=ops.SILU)  # noqa: E731
        for q in paths:
            ops.set_conv_path(q[0])
            ops.set_conv_option(0, q[1])
            ops.set_conv_option(2, q[2])
            ops.set_conv_option(3, q[3])
            ops.SPLITK_ALLOWED = bool(q[4])
            ops.set_conv_option(4, q[5])
            outs[q] = fn()
        for _ in range(3):
            for q in paths:
                ops.set_conv_path(q[0])
                ops.set_conv_option(0, q[1])
                ops.set_conv_option(2, q[2])
                ops.set_conv_option(3, q[3])
                ops.SPLITK_ALLOWED = bool(q[4])
                ops.set_conv_option(4, q[5])
                times[q].append(bench(fn, args.reps))
        flops = 2.0 * B * (H // stride) * (W // stride) * cout * cin * k * k
        r = dict(name=name)
        for q in paths:
            r["tf_" + "".join(f"{k}{v}" for k, v in zip("pefzkt", q))] = round(flops / min(times[q]) / 1e12, 1)
        r["identical"] = all(torch.equal(outs[paths[0]], outs[q]) for q in paths if q[4] == 0)
        r["max_diff_splitk"] = max([(outs[paths[0]].float() - outs[q].float()).abs().max().item()
                                    for q in paths if q[4] == 1] or [0.0])
        print(json.dumps(r), flush=True)
        res.append(r)
    ops.set_conv_path(2)
    ops.set_conv_option(0, 1)
    ops.set_conv_option(2, 0)
    ops.set_conv_option(3, 1)
    ops.SPLITK_ALLOWED = False
    ops.set_conv_option(4, -1)


if __name__ == "__main__":
    main()
