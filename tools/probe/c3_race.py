"""Locate the run-to-run nondeterminism of config 3 (B=8 1024^2 bf16): repeat the VAE encoder and
the compressor's g_a / hyper encoder eagerly on fixed inputs and report which stage's output
changes between repeats, with the flash VAE attention on and off."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import ops  # noqa: E402
from rdeic_amd import weights as W  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import synth_image  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
R = int(sys.argv[3]) if len(sys.argv) > 3 else 10
imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
pc = m.preprocess_model


def diff_imgs(a, b):
    return [int((a[i] != b[i]).sum().item()) for i in range(a.shape[0])]


with torch.no_grad():
    for flash in (True, False):
        ops.VAE_FLASH_ATTENTION = flash
        h0 = m.encode_images_nhwc(imgs).clone()
        bad = 0
        for r in range(R):
            h = m.encode_images_nhwc(imgs)
            d = diff_imgs(h0, h)
            if any(d):
                bad += 1
                print(f"flash={flash} encoder run {r}: elements differing per image {d}", flush=True)
        print(f"flash={flash}: encoder differs in {bad}/{R} repeats", flush=True)
    ops.VAE_FLASH_ATTENTION = True
    y0 = pc._seq(pc.g_a, h0).clone()
    z0 = pc._seq(pc.hyper_enc, y0).clone()
    bad_y = bad_z = 0
    for r in range(R):
        y = pc._seq(pc.g_a, h0)
        z = pc._seq(pc.hyper_enc, y0)
        dy, dz = diff_imgs(y0, y), diff_imgs(z0, z)
        bad_y += any(dy)
        bad_z += any(dz)
        if any(dy) or any(dz):
            print(f"g_a run {r}: y diffs {dy}; hyper_enc z diffs {dz}", flush=True)
    print(f"g_a differs in {bad_y}/{R}, hyper_enc in {bad_z}/{R}", flush=True)
