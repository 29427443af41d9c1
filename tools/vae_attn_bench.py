"""VAE AttnBlock attention (single head, d = 512, bf16): the flash kernel (rdeic_attention, dh 512)
against the materialised GEMM -> softmax -> GEMM path, at config 2's (16 x 64^2 latents) and config
3's (8 x 128^2) shapes. TFLOP/s = 4 B L^2 d / time (HIP events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


def main():
    C = 512
    for B, L in ((16, 4096), (8, 16384)):
        qkv = torch.randn(B * L, 3 * C, device="cuda").to(torch.bfloat16)
        q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
        o1, o2 = (torch.empty(B * L, C, dtype=torch.bfloat16, device="cuda") for _ in range(2))
        flops = 4.0 * B * L * L * C
        t_flash = timeit(lambda: ops.attention(q, k, v, o1, batch=B, heads=1, lq=L, lk=L, dh=C, scale=C ** -0.5))
        t_mat = timeit(lambda: ops.attention_single_head_materialized(q, k, v, o2, batch=B, length=L, dim=C,
                                                                      scale=C ** -0.5))
        print(json.dumps({"B": B, "L": L, "flash_ms": round(t_flash, 3), "flash_tflops": round(flops / t_flash / 1e9, 1),
                          "materialized_ms": round(t_mat, 3), "materialized_tflops": round(flops / t_mat / 1e9, 1),
                          "max_abs_diff": (o1.float() - o2.float()).abs().max().item()}), flush=True)


if __name__ == "__main__":
    main()
