"""Config 3 (8 x 1024^2, bf16) determinism probe: is the compress path run-to-run / plan-replay
stable? Compares the VAE feature h of repeated eager runs (per image), the eager bodies of two
runs, and the plan record vs replay bodies."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import weights as W  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import synth_image  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
with torch.no_grad():
    hs = [m.encode_images_nhwc(imgs) for _ in range(3)]
    torch.cuda.synchronize()
    for i in range(B):
        d = [(hs[0][i].float() - h[i].float()).abs().max().item() for h in hs[1:]]
        print(f"h image {i}: max |diff| run1/run2 vs run0 {d}", flush=True)
    solo = m.encode_images_nhwc(imgs[6:7])
    print("h image 6 solo vs batch:", (solo[0].float() - hs[0][6].float()).abs().max().item(), flush=True)
    m.use_plans = False
    e1 = m.preprocess_model.compress(hs[0])
    e2 = m.preprocess_model.compress(hs[0])
    print("eager compress bodies equal per image:", [a == b for a, b in zip(e1, e2)], flush=True)
    m.use_plans = True
    p1 = m.compress_images(imgs)
    p2 = m.compress_images(imgs)
    p3 = m.compress_images(imgs)
    print("plan record vs replay:", [a == b for a, b in zip(p1, p2)], flush=True)
    print("replay vs replay:", [a == b for a, b in zip(p2, p3)], flush=True)
    from rdeic_amd import bitstream
    eb = [bitstream.pack_body(o["shape"], o["strings"]) for o in e1]
    print("eager (from h run0) vs plan record:", [a == b for a, b in zip(eb, p1)], flush=True)
