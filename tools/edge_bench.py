"""Times the VAE edge convs (conv_edge.hip) and the fused GroupNorm finalize + apply on the bench's shapes,
each against the path it replaced (same process, alternating, HIP events on the launch stream).

  python tools/edge_bench.py [REPS] [only]   (GPU box) -> one JSON line per case
  only: the edge kernels alone, no replaced paths, no GroupNorm cases (PMC runs)
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402


def timed(fn, reps):
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
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    only = len(sys.argv) > 2 and sys.argv[2] == "only"
    torch.manual_seed(0)
    n, h, w = 16, 512, 512
    # conv_in: 8 (3 real) -> 128, with the GroupNorm statistics of the output
    x8 = torch.zeros(n, h, w, 8, device="cuda")
    x8[..., :3] = torch.rand(n, h, w, 3, device="cuda") * 2 - 1
    x8 = x8.to(torch.bfloat16)
    wt = torch.zeros(128, 8, 3, 3)
    wt[:, :3] = torch.randn(128, 3, 3, 3) / math.sqrt(27)
    p_in = ops.ConvParams.pack(wt, torch.randn(128) * 0.1, pad=1)
    # norm -> SiLU -> conv_out: 128 -> 3, fp32 out
    xh = torch.randn(n, h, w, 128, device="cuda").to(torch.bfloat16)
    ab = ops.group_norm_ab(xh, torch.ones(128, device="cuda"), torch.zeros(128, device="cuda"), 32, 1e-6)
    p_out = ops.ConvParams.pack(torch.randn(3, 128, 3, 3) / math.sqrt(1152), torch.randn(3), pad=1)
    cases = {
        "conv_in 16x512^2 8->128 +stats": (lambda: ops.conv2d(x8, p_in, stats=True),
                                           n * h * w * (8 + 128) * 2),
        "norm+swish+conv_out 16x512^2 128->3": (lambda: ops.conv2d(xh, p_out, gn=ab, gn_silu=True, out_f32=True),
                                                n * h * w * (128 * 2 + 3 * 4)),
    }
    for name, (fn, byts) in cases.items():
        res = {}
        modes = (1, 0)
        if only:
            prev = ops.set_edge_conv(1)
            ms = timed(fn, reps)
            ops.set_edge_conv(prev)
            print(json.dumps({"case": name, "ms": round(ms, 4)}), flush=True)
            continue
        for _ in range(2):
            for edge in modes:
                prev = ops.set_edge_conv(edge)
                try:
                    ms = timed(fn, reps)
                finally:
                    ops.set_edge_conv(prev)
                res.setdefault(edge, []).append(ms)
        e, o = min(res[1]), min(res[0])
        extra = {f"mode{m}_ms": round(min(v), 4) for m, v in res.items() if m > 1}
        print(json.dumps({"case": name, **extra, "edge_ms": round(e, 4), "edge_TBps": round(byts / e / 1e9, 2),
                          "replaced_ms": round(o, 4), "replaced_TBps": round(byts / o / 1e9, 2),
                          "algorithmic_bytes": byts}), flush=True)
    if only:
        return
    # fused GroupNorm finalize + apply vs parts_ab + apply (the UNet's 16^2 / 8^2 GroupNorms)
    for (hh, c0, c1) in ((16, 1280, 0), (16, 1280, 1280), (8, 1280, 0), (8, 1280, 1280), (16, 640, 640)):
        xa = torch.randn(n, hh, hh, 256, device="cuda").to(torch.bfloat16)
        wa = torch.randn(c0, 256, 1, 1) / 16
        ya = ops.conv2d(xa, ops.ConvParams.pack(wa, None), stats=True)
        yb = ops.conv2d(xa, ops.ConvParams.pack(torch.randn(c1, 256, 1, 1) / 16, None), stats=True) if c1 else None
        g, b = torch.ones(c0 + c1, device="cuda"), torch.zeros(c0 + c1, device="cuda")
        pc = ops.ConvParams.pack(torch.randn(64, c0 + c1, 1, 1) / 30, None)
        xin = torch.empty(n, hh, hh, c0 + c1, dtype=torch.bfloat16, device="cuda")

        def fused():
            ab_d = ops.group_norm_ab(ya, g, b, 32, 1e-5, x2=yb, defer=True)
            p0, pc0, p1, cc1, n_, hw_, groups, eps, gamma, beta = ab_d._rdeic_pending
            ops.call("rdeic_groupnorm_parts_apply", p0.data_ptr(), pc0, ops._ptr(p1), cc1, ya.data_ptr(),
                     ops.pix_ld(ya), ops._ptr(yb), ops.pix_ld(yb) if yb is not None else 0, n_, hw_, groups, eps,
                     gamma.data_ptr(), beta.data_ptr(), 1, ab_d.data_ptr(), xin.data_ptr(), ops.pix_ld(xin),
                     ops.stream_ptr())

        def two():
            ab_n = ops.group_norm_ab(ya, g, b, 32, 1e-5, x2=yb)
            ops.group_norm_apply(ya, ab_n, True, out=xin[..., :c0])
            if yb is not None:
                ops.group_norm_apply(yb, ab_n[:, c0:], True, out=xin[..., c0:])

        tf = min(timed(fused, reps) for _ in range(2))
        tt = min(timed(two, reps) for _ in range(2))
        print(json.dumps({"case": f"groupnorm {n}x{hh}^2 {c0}+{c1}", "fused_us": round(tf * 1e3, 2),
                          "two_launch_us": round(tt * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
