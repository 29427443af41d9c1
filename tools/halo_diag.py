"""Where the halo conv's time goes, per VAE shape (B=16): the full ResnetBlock form (GroupNorm +
SiLU in LDS, residual, fused output statistics) against the same kernel without the transform
(conv3x3_halo_kernel<false>, option 6 = 2) and without the epilogue extras.
  python tools/halo_diag.py [HxCINxCOUT ...]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from tools.halo_bench import SHAPES, timeit  # noqa: E402


def main():
    only = sys.argv[1:]
    for n, h, w, cin, cout in SHAPES:
        if only and f"{h}x{cin}x{cout}" not in only:
            continue
        x = torch.randn(n, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, 3, 3, device="cuda") / math.sqrt(cin * 9)
        p = ops.ConvParams.pack(wt, torch.zeros(cout, device="cuda"), pad=1)
        ab = ops.group_norm_ab(x, torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda"), 32, 1e-6)
        res = torch.randn(n, h, w, cout, device="cuda").to(torch.bfloat16)
        out = torch.empty(n, h, w, cout, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * n * h * w * cout * 9 * cin
        ops.set_halo_conv(1)
        full = timeit(lambda: ops.conv2d(x, p, gn=ab, gn_silu=True, res=res, out=out, stats=True))
        gn_only = timeit(lambda: ops.conv2d(x, p, gn=ab, gn_silu=True, out=out))
        gn_res = timeit(lambda: ops.conv2d(x, p, gn=ab, gn_silu=True, res=res, out=out))
        gn_st = timeit(lambda: ops.conv2d(x, p, gn=ab, gn_silu=True, out=out, stats=True))
        ops.set_halo_conv(2)
        plain = timeit(lambda: ops.conv2d(x, p, out=out))
        plain_epi = timeit(lambda: ops.conv2d(x, p, res=res, out=out, stats=True))
        ops.set_halo_conv(0)
        tile = timeit(lambda: ops.conv2d(x, p, out=out))
        ops.set_halo_conv(1)
        tf = lambda ms: flops / ms / 1e9  # noqa: E731
        print(f"{h}x{cin}x{cout}: full {full:.3f} ms ({tf(full):.0f} TF) | gn, no res/stats {gn_only:.3f} "
              f"({tf(gn_only):.0f}) | no gn {plain:.3f} ({tf(plain):.0f}) | no gn + res/stats {plain_epi:.3f} "
              f"({tf(plain_epi):.0f}) | im2col tile, no gn {tile:.3f} ({tf(tile):.0f}) | gn + res only {gn_res:.3f} "
              f"| gn + stats only {gn_st:.3f}", flush=True)


if __name__ == "__main__":
    main()
