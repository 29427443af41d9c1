"""d = 512 flash attention forms A/B (rdeic_set_conv_option(8, v): 1 one wave per 16 queries,
2 wave pairs splitting d over 32 queries) at config 2's (16 x 64^2) and config 3's (8 x 128^2)
shapes: max |difference| between the forms and against torch fp32, TFLOP/s interleaved."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402


def timeit(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    torch.manual_seed(0)
    C = 512
    for B, L in ((16, 4096), (8, 16384), (2, 1024)):
        q, k, v = (torch.randn(B * L, C, device="cuda").to(torch.bfloat16) for _ in range(3))
        outs, ms = {}, {1: [], 2: []}
        for form in (1, 2):
            ops.set_conv_option(8, form)
            o = torch.empty(B * L, C, device="cuda", dtype=torch.bfloat16)
            ops.attention(q, k, v, o, batch=B, heads=1, lq=L, lk=L, dh=C, scale=C ** -0.5)
            torch.cuda.synchronize()
            outs[form] = o
        for _ in range(3):
            for form in (1, 2):
                ops.set_conv_option(8, form)
                ms[form].append(timeit(lambda: ops.attention(q, k, v, outs[form], batch=B, heads=1, lq=L, lk=L, dh=C,
                                                             scale=C ** -0.5)))
        ops.set_conv_option(8, 2)
        flops = 4.0 * B * L * L * C
        nb = min(B, 2)
        q3, k3, v3 = (t.view(B, L, C)[:nb].float() for t in (q, k, v))
        ref = torch.softmax((q3 @ k3.transpose(1, 2)) * C ** -0.5, dim=-1) @ v3
        r = {"B": B, "L": L,
             "tf_form1": round(flops / min(ms[1]) / 1e9, 1), "tf_form2": round(flops / min(ms[2]) / 1e9, 1),
             "max_diff_forms": (outs[1].float() - outs[2].float()).abs().max().item(),
             "max_err_form2_vs_fp32": (outs[2].view(B, L, C)[:nb].float() - ref).abs().max().item(),
             "max_err_form1_vs_fp32": (outs[1].view(B, L, C)[:nb].float() - ref).abs().max().item()}
        print(json.dumps(r), flush=True)
        del q, k, v, outs, ref, q3, k3, v3
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
