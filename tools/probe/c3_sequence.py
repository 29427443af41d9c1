"""Config-3 test sequence probe: tests/test_config3_gpu.py's bf16 B=8 order of calls (compress B=8,
compress B=1, decompress B=8, decompress B=1, codec_images B=8), then which of the bodies deviate:
the first (recording) call, the later replays, or an eager run."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import weights as W  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import sampler_noise, synth_context, synth_image  # noqa: E402

S, B = 1024, 8
steps = [s for s in sys.argv[1:]] or ["solo", "dec", "dec1", "codec"]
imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
with torch.no_grad():
    bodies = m.compress_images(imgs)
    b_again = m.compress_images(imgs)
    print("record vs first replay:", [a == b for a, b in zip(bodies, b_again)], flush=True)
    if "solo" in steps:
        solo = m.compress_images(imgs[1:2])
        print("solo == batch[1]:", solo[0] == bodies[1], flush=True)
        print("after solo, replay:", [a == b for a, b in zip(bodies, m.compress_images(imgs))], flush=True)
    if "dec" in steps:
        c_b, h_b = m.decompress_bodies(bodies)
        print("after decompress B=8, replay:", [a == b for a, b in zip(bodies, m.compress_images(imgs))], flush=True)
    if "dec1" in steps:
        c_s, h_s = m.decompress_bodies(bodies[1:2])
        print("after decompress B=1, replay:", [a == b for a, b in zip(bodies, m.compress_images(imgs))], flush=True)
    if "codec" in steps:
        ctx = synth_context().cuda()
        _, noise = sampler_noise((B, 4, S // 8, S // 8), 231)
        out, bodies2 = m.codec_images(imgs, ctx, noise, steps=5)
        print("codec_images bodies:", [a == b for a, b in zip(bodies, bodies2)], flush=True)
        print("after codec, replay:", [a == b for a, b in zip(bodies, m.compress_images(imgs))], flush=True)
    m.use_plans = False
    eb = m.compress_images(imgs)
    print("eager vs first:", [a == b for a, b in zip(bodies, eb)], flush=True)
