"""Time the VAE conv_out shape (128 -> 3, GN + SiLU prologue) in isolation."""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

x = torch.randn(16, 512, 512, 128, device="cuda").to(torch.bfloat16)
w = torch.randn(3, 128, 3, 3, device="cuda") / math.sqrt(128 * 9)
p = ops.ConvParams.pack(w, torch.randn(3, device="cuda"), pad=1)
gamma, beta = torch.rand(128, device="cuda") + 0.5, torch.randn(128, device="cuda")
ab = ops.group_norm_ab(x, gamma, beta, 32, 1e-6)
for _ in range(3):
    ops.conv2d(x, p, gn=ab, gn_silu=True, out_f32=True)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(10):
    ops.conv2d(x, p, gn=ab, gn_silu=True, out_f32=True)
torch.cuda.synchronize()
print("conv_out ms", (time.perf_counter() - t) / 10 * 1e3)
