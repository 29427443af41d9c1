"""smoke(): one small end-to-end codec invocation on cuda:0, checked against the oracle.

Runs golden image 0 (128x128, 2 relay DDIM steps) through the HIP path in fp32 and checks
(1) the bitstream body is byte-identical to the reference fixture and to oracle/model_ref.py,
(2) the reconstructed uint8 image is within 1 level of the oracle's (same as the reference's)."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "e2e_128.npz")


def run_smoke():
    assert torch.cuda.is_available(), "smoke() needs a GPU"
    from rdeic_amd import _lib
    _lib.load()  # loud failure if the HIP library is missing
    from rdeic_amd.rdeic import RDEIC
    from oracle import model_ref as M

    g = np.load(GOLDEN)
    img = g["img0_in"]
    noise = torch.from_numpy(g["img0_noise"])
    ctx = torch.from_numpy(g["context"])
    model = RDEIC(compute_dtype=torch.float32).init_synthetic()
    out, bodies = model.codec_images(torch.from_numpy(img[None]).cuda(), ctx.cuda(), noise, steps=2)
    torch.cuda.synchronize()
    out = out.cpu().numpy()[0]

    sd = M.synthetic_state_dict()
    ref_img, ref_body = M.codec_image(sd, M.Tables(), img, ctx, noise, steps=2, coder="c")
    assert bytes(bodies[0]) == ref_body == g["img0_file"].tobytes(), "bitstream differs from oracle"
    diff = np.abs(out.astype(np.int32) - ref_img.astype(np.int32)).max()
    assert diff <= 1, f"reconstruction differs from oracle by {diff} levels"
    print(f"smoke ok: {len(ref_body)} byte body identical, max pixel diff {diff}")
