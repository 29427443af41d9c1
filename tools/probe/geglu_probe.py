"""GEGLU projection cost split: fused epilogue vs the plain projection (same GEMM, no GEGLU) vs
projection + stand-alone rdeic_geglu, per tile, at the UNet's GEGLU shapes (B=16, bf16)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import ops  # noqa: E402


def t_ms(fn, reps=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


torch.manual_seed(0)
for M, cin, inner in [(65536, 320, 1280), (16384, 640, 2560), (4096, 1280, 5120)]:
    x = torch.randn(1, M, 1, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(2 * inner, cin, 1, 1, device="cuda") / math.sqrt(cin)
    b = torch.randn(2 * inner, device="cuda")
    p = ops.ConvParams.pack(w, b)
    out_g = torch.empty(1, M, 1, inner, device="cuda", dtype=torch.bfloat16)
    out_p = torch.empty(1, M, 1, 2 * inner, device="cuda", dtype=torch.bfloat16)
    fl = 2.0 * M * cin * 2 * inner
    for tile in (None, 34, 32, 33, 25, 29):
        ops.FORCE_TILE = tile
        tg = t_ms(lambda: ops.conv2d(x, p, geglu=True, out=out_g))
        tp = t_ms(lambda: ops.conv2d(x, p, out=out_p))
        ts = t_ms(lambda: ops.geglu(out_p.view(M, 2 * inner)))
        print(f"M{M} {cin}->{2 * inner} tile {tile}: fused {tg * 1e3:7.1f} us ({fl / tg / 1e9:6.1f} TF/s)  "
              f"plain {tp * 1e3:7.1f} us ({fl / tp / 1e9:6.1f})  geglu-alone {ts * 1e3:6.1f} us", flush=True)
    ops.FORCE_TILE = None
