"""Compare conv paths against each other and a torch fp32 reference on one shape (debug aid)."""
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

torch.manual_seed(0)
for (B, H, W, cin, cout) in [(2, 64, 64, 128, 128), (2, 32, 32, 512, 512), (4, 16, 16, 320, 320)]:
    x = torch.randn(B, H, W, cin, device="cuda").to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, device="cuda") / math.sqrt(cin * 9)
    b = torch.randn(cout, device="cuda")
    p = ops.ConvParams.pack(w, b, pad=1)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.to(torch.bfloat16).float(), b, padding=1).permute(0, 2, 3, 1)
    outs = {}
    for path in (0, 1, 2):
        for pf in (0, 1):
            ops.set_conv_path(path)
            ops.set_conv_option(2, pf)
            o = ops.conv2d(x, p, out_f32=True)
            outs[(path, pf)] = o
            print((B, H, W, cin, cout), "path", path, "pf2", pf, "max|d| vs ref", (o - ref).abs().max().item())
    base = outs[(1, 0)]
    for k, o in outs.items():
        print("   ", k, "identical to path1:", torch.equal(o, base), "max diff", (o - base).abs().max().item())
ops.set_conv_path(2)
ops.set_conv_option(2, 0)
