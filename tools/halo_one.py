"""One conv shape, a few launches of the halo kernel and of the im2col tile (PMC target):
  python tools/halo_one.py [H] [cin] [cout] [reps]"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402

H = int(sys.argv[1]) if len(sys.argv) > 1 else 512
cin = int(sys.argv[2]) if len(sys.argv) > 2 else 128
cout = int(sys.argv[3]) if len(sys.argv) > 3 else 128
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 4
x = torch.randn(16, H, H, cin, device="cuda").to(torch.bfloat16)
w = torch.randn(cout, cin, 3, 3, device="cuda") / math.sqrt(cin * 9)
p = ops.ConvParams.pack(w, torch.zeros(cout, device="cuda"), pad=1)
ab = ops.group_norm_ab(x, torch.ones(cin, device="cuda"), torch.zeros(cin, device="cuda"), 32, 1e-6)
out = torch.empty(16, H, H, cout, device="cuda", dtype=torch.bfloat16)
for mode in (1, 0):
    ops.set_halo_conv(mode)
    for _ in range(reps):
        ops.conv2d(x, p, gn=ab, gn_silu=True, out=out)
torch.cuda.synchronize()
