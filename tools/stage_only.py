"""Run one pipeline stage repeatedly (for rocprofv3 --stats attribution): unet | vae_dec | vae_enc."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import sampler_noise, synth_context, synth_image  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--stage", default="unet")
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
B, S = 16, 512
model = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
ctx = synth_context().cuda()
c_lat = torch.randn(B, S // 8, S // 8, 4, device="cuda")
hint = torch.randn(B, S // 8, S // 8, 256, device="cuda").to(torch.bfloat16)
nz = torch.randn(B, S // 8, S // 8, 4, device="cuda")
for _ in range(args.reps):
    if args.stage == "unet":
        model.relay_sample_nhwc(c_lat, hint, ctx, nz, 2)
    elif args.stage == "vae_dec":
        model.decode_nhwc(c_lat)
    else:
        model.encode_images_nhwc(imgs)
torch.cuda.synchronize()
