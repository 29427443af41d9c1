"""Same-process A/B of the 256-channel halo conv (rdeic_set_conv_option(10, 1)) against halo8 / the 4-row form on
the VAE ResnetBlock shapes with cout >= 256 (B = 16, GroupNorm + SiLU input, residual, fused statistics),
interleaved over REPS rounds. Prints ms and TFLOP/s per variant (median over rounds).
usage (GPU box): python tools/halo256_ab.py [REPS]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

SHAPES = [(16, 256, 256, 256, 256, True), (16, 256, 256, 256, 256, False), (16, 128, 128, 512, 512, True),
          (16, 128, 128, 512, 512, False), (16, 64, 64, 512, 512, True), (16, 256, 256, 512, 256, False),
          (16, 256, 256, 128, 256, False), (16, 128, 128, 256, 512, False)]


def timeit(fn, reps=8):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    ops.HALO_MAX_C = 512
    for n, h, w, cin, cout, use_res in SHAPES:
        x = torch.randn(n, h, w, cin, device="cuda").to(torch.bfloat16)
        wt = torch.randn(cout, cin, 3, 3, device="cuda") / math.sqrt(cin * 9)
        p = ops.ConvParams.pack(wt, torch.zeros(cout, device="cuda"), pad=1)
        ab = ops.group_norm_ab(x, torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda"), 32, 1e-6)
        res = torch.randn(n, h, w, cout, device="cuda").to(torch.bfloat16) if use_res else None
        out = torch.empty(n, h, w, cout, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * n * h * w * cout * 9 * cin
        r = {"halo256": [], "halo8": [], "halo4": []}
        for _ in range(rounds):
            for name, o10, o9 in (("halo256", 1, 1), ("halo8", 0, 1), ("halo4", 0, 0)):
                p10, p9 = ops.set_conv_option(10, o10), ops.set_conv_option(9, o9)
                r[name].append(timeit(lambda: ops.conv2d(x, p, gn=ab, gn_silu=True, res=res, out=out, stats=True)))
                ops.set_conv_option(10, p10)
                ops.set_conv_option(9, p9)
        med = {k: sorted(v)[len(v) // 2] for k, v in r.items()}
        print(f"{n}x{h}x{w} {cin}->{cout}{' +res' if use_res else ''}: " +
              ", ".join(f"{k} {v:.3f} ms ({flops / v / 1e9:.0f} TF)" for k, v in med.items()), flush=True)


if __name__ == "__main__":
    main()
