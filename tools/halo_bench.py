"""A/B of the VAE ResnetBlock conv with a GroupNorm + SiLU input at the bench's shapes (B=16):
materialised (rdeic_groupnorm_apply + the tiled im2col conv) vs the halo conv (affine in LDS).
Prints ms per call and TFLOP/s of the conv FLOPs (the apply's bytes counted as time only)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

SHAPES = [(16, 512, 512, 128, 128), (16, 512, 512, 256, 128), (16, 256, 256, 128, 256), (16, 256, 256, 256, 256),
          (16, 128, 128, 256, 512), (16, 128, 128, 512, 512), (16, 64, 64, 512, 512)]


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


# UNet-ResBlock-like shapes the halo kernel can take (64-pixel rows, cout % 128): the in_layers conv
# carries the timestep embedding (emb); the UNet's own widths (320 / 640 / 1280 at 64^2..8^2) need a
# 160-wide N tile and narrower image rows, so these bracket what a fused UNet ResBlock conv would gain
SHAPES_UNET = [(16, 64, 64, 256, 256), (16, 64, 64, 384, 384), (16, 64, 64, 512, 512)]


def main():
    only = sys.argv[1:]
    unet = "unet" in only
    for n, h, w, cin, cout in (SHAPES_UNET if unet else SHAPES):
        if only and not unet and f"{h}x{cin}x{cout}" not in only:
            continue
        x = torch.randn(n, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, 3, 3, device="cuda") / math.sqrt(cin * 9)
        p = ops.ConvParams.pack(wt, torch.zeros(cout, device="cuda"), pad=1)
        gamma, beta = torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda")
        ab = ops.group_norm_ab(x, gamma, beta, 32, 1e-6)
        res = torch.randn(n, h, w, cout, device="cuda").to(torch.bfloat16)
        out = torch.empty(n, h, w, cout, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * n * h * w * cout * 9 * cin
        emb = torch.randn(n, cout, device="cuda") if unet else None
        r = {}
        for mode in (0, 1):
            ops.set_halo_conv(mode)
            ms = timeit(lambda: ops.conv2d(x, p, gn=ab, gn_silu=True, emb=emb, res=None if unet else res, out=out,
                                           stats=True))
            r[mode] = ms
        ops.set_halo_conv(1)
        print(f"{n}x{h}x{w} {cin}->{cout}{' +emb' if unet else ''}: materialised {r[0]:.3f} ms ({flops / r[0] / 1e9:.0f} TF eff), "
              f"halo {r[1]:.3f} ms ({flops / r[1] / 1e9:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
