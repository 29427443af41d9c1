"""Attention kernel micro-benchmark on the UNet shapes (bf16, batch 16): generic (0), register-staged
dh=64 (1) and LDS-DMA dh=64 (2) kernels."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

SHAPES = [  # name, B, heads, lq, lk, dh, kv_bcast
    ("self4096", 16, 5, 4096, 4096, 64, False),
    ("self1024", 16, 10, 1024, 1024, 64, False),
    ("self256", 16, 20, 256, 256, 64, False),
    ("cross4096", 16, 5, 4096, 77, 64, True),
    ("self16384_cfg3", 8, 5, 16384, 16384, 64, False),
    ("ctrl16_self4096", 16, 4, 4096, 4096, 16, False),
    ("ctrl16_self16384_cfg3", 8, 4, 16384, 16384, 16, False),
]


# rdeic_set_conv_option(1, mode) values timed for dh = 64 (argv[1], comma-separated; default 0,1,2)
MODES = tuple(int(v) for v in sys.argv[1].split(",")) if len(sys.argv) > 1 else (0, 1, 2)


def bench(fn, reps):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    torch.manual_seed(0)
    for name, B, H, lq, lk, dh, bc in SHAPES:
        q = torch.randn(B, lq, H * dh, device="cuda").to(torch.bfloat16)
        kb = 1 if bc else B
        k = torch.randn(kb, lk, H * dh, device="cuda").to(torch.bfloat16)
        v = torch.randn(kb, lk, H * dh, device="cuda").to(torch.bfloat16)
        o = torch.empty_like(q)

        def fn():
            ops.attention(q.view(-1, H * dh), k.view(-1, H * dh), v.view(-1, H * dh), o.view(-1, H * dh), batch=B,
                          heads=H, lq=lq, lk=lk, dh=dh, scale=dh ** -0.5, kv_bcast=bc)
            return o.clone()
        res = {"name": name}
        outs = {}
        modes = MODES if dh == 64 else (2,)
        for mode in modes:
            ops.set_conv_option(1, mode)
            outs[mode] = fn()
            t = min(bench(fn, 5) for _ in range(3))
            flops = 4.0 * B * H * lq * lk * dh
            res[f"tflops_k{mode}"] = round(flops / t / 1e12, 1)
        # fp32 reference on the first 2 images
        qf, kf, vf = q[:2].float(), k[:min(2, kb)].float(), v[:min(2, kb)].float()
        qh = qf.view(2, lq, H, dh).transpose(1, 2)
        kh = kf.view(-1, lk, H, dh).transpose(1, 2)
        vh = vf.view(-1, lk, H, dh).transpose(1, 2)
        ref = torch.softmax(qh @ kh.transpose(-1, -2) * dh ** -0.5, -1) @ vh
        ref = ref.transpose(1, 2).reshape(2, lq, H * dh)
        for mode in modes:
            res[f"maxerr_k{mode}"] = round((outs[mode][:2].float() - ref).abs().max().item(), 4)
        print(json.dumps(res), flush=True)
    ops.set_conv_option(1, 2)


if __name__ == "__main__":
    main()
