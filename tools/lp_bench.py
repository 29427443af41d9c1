"""Persistent short-K linear (option 12) against the LDS-DMA tiles on the bench's transformer projections.

For each shape: us per launch with option 12 = 0 (the tile table / heuristic) and = 2 (linear_persist_kernel),
min over 3 runs of 10 launches each (HIP events on the current stream), bf16, random weights.
usage (GPU box): python tools/lp_bench.py > out.jsonl"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from rdeic_amd.params import ParamStore  # noqa: E402

SHAPES = [  # rows, cin, cout, geglu, ln
    (65536, 320, 2560, True, True), (16384, 640, 5120, True, True), (4096, 1280, 10240, True, True),
    (65536, 320, 960, False, True), (16384, 640, 1920, False, True), (4096, 1280, 3840, False, True),
    (65536, 320, 320, False, True), (16384, 640, 640, False, True), (4096, 1280, 1280, False, True),
]


OPTS = tuple(int(v) for v in sys.argv[1].split(",")) if len(sys.argv) > 1 else (0, 2)


def main():
    torch.manual_seed(0)
    for rows, cin, cout, geglu, ln in SHAPES:
        x = torch.randn(rows, cin, device="cuda").to(torch.bfloat16)
        st = ParamStore(torch.bfloat16, "cuda")
        st.shapes["l0.weight"], st.shapes["l0.bias"] = (cout, cin), (cout,)
        st.t["l0.weight"] = torch.randn(cout, cin, device="cuda") / math.sqrt(cin)
        st.t["l0.bias"] = torch.randn(cout, device="cuda") * 0.1
        ms = None
        if ln:
            st.shapes["ln.weight"] = st.shapes["ln.bias"] = (cin,)
            st.t["ln.weight"], st.t["ln.bias"] = torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda")
            p = st.conv_ln(["l0"], "ln", geglu=geglu)
            ms = ops.layer_norm_rowstats(x)
        else:
            p = st.conv_geglu("l0") if geglu else st.conv("l0")
        res = {"shape": [rows, cin, cout], "geglu": geglu, "ln": ln}
        for opt in OPTS:
            # opt < 20: option 12 (persistent linear) value; opt >= 20: that LDS-DMA tile forced, option 12 off
            prev = ops.set_conv_option(12, opt if opt < 20 else 0)
            ops.FORCE_TILE = opt if opt >= 20 else None
            try:
                y = ops.linear(x, p, geglu=geglu, images=1, ln_rows=ms)
                best = 1e9
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(10):
                        ops.linear(x, p, geglu=geglu, images=1, ln_rows=ms, out=y)
                    e1.record()
                    torch.cuda.synchronize()
                    best = min(best, e0.elapsed_time(e1) / 10 * 1e3)
            finally:
                ops.set_conv_option(12, prev)
                ops.FORCE_TILE = None
            res[f"us_opt{opt}"] = round(best, 1)
            res[f"tflops_opt{opt}"] = round(2.0 * rows * cin * cout / (best * 1e-6) / 1e12, 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
