"""Transformer linears of the UNet at the bench's shapes (B=16, 512^2 images), every LDS-DMA tile,
timed as a captured hipGraph of 20 launches (no host launch overhead in the figure): per-launch us,
TFLOP/s and the effective HBM rate of the algorithmic bytes (A + W + out [+ residual])."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from rdeic_amd.params import ParamStore  # noqa: E402

# name, rows, K, N, residual, geglu
SHAPES = [("qk320@64", 65536, 320, 320, True, False), ("qkv320@64", 65536, 320, 960, False, False),
          ("geglu320@64", 65536, 320, 2560, False, True), ("ff1280->320@64", 65536, 1280, 320, True, False),
          ("o640@32", 16384, 640, 640, True, False), ("geglu640@32", 16384, 640, 5120, False, True),
          ("ff2560->640@32", 16384, 2560, 640, True, False), ("o1280@16", 4096, 1280, 1280, True, False),
          ("geglu1280@16", 4096, 1280, 10240, False, True)]
TILES = (-1, 21, 22, 24, 25, 26, 27, 30, 31, 32, 33, 34, 36, 37, 38)


def main():
    only = [a for a in sys.argv[1:] if a != "--ln"]
    ln = "--ln" in sys.argv[1:]  # the model's form: LayerNorm folded into the projection (ParamStore.conv_ln)
    torch.manual_seed(0)
    for name, M, K, N, res, geglu in SHAPES:
        if only and not any(o in name for o in only):
            continue
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = torch.randn(N, K, device="cuda") / math.sqrt(K)
        b = torch.randn(N, device="cuda") * 0.1
        st = ParamStore(torch.bfloat16, "cuda")
        st.shapes["l.weight"], st.shapes["l.bias"] = (N, K), (N,)
        st.t["l.weight"], st.t["l.bias"] = w, b
        lnr = None
        if ln:
            st.shapes["n.weight"], st.shapes["n.bias"] = (K,), (K,)
            st.t["n.weight"], st.t["n.bias"] = 1 + 0.1 * torch.randn(K, device="cuda"), 0.1 * torch.randn(K, device="cuda")
            p = st.conv_ln(["l"], "n", geglu=geglu)
            lnr = ops.layer_norm_rowstats(x)
        else:
            p = st.conv_geglu("l") if geglu else st.conv("l")
        nout = N // 2 if geglu else N
        r = torch.randn(M, nout, device="cuda").to(torch.bfloat16) if res else None
        out = torch.empty(M, nout, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * M * K * N
        bytes_ = 2.0 * (M * K + N * K + M * nout * (2 if res else 1))
        row = {"name": name + ("+ln" if ln else "")}
        for t in TILES:
            ops.FORCE_TILE = t if t >= 0 else None
            try:
                fn = lambda: ops.linear(x, p, res=r, out=out, geglu=geglu, images=16, ln_rows=lnr)  # noqa: E731
                fn()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(20):
                        fn()
                g.replay()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / 20
                row[f"t{t}"] = [round(us, 1), round(flops / us / 1e6), round(bytes_ / us / 1e3)]
            except Exception as e:  # a tile that cannot run this shape
                row[f"t{t}"] = str(e)[:40]
            finally:
                ops.FORCE_TILE = None
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
