"""Golden vector of config 3's relay denoiser at 1024x1024 (latent 128x128), produced by the
REFERENCE's own modules on CPU, fp32: ONE NoiseEstimator call (model/rdeic.py:174-212: control
branch + frozen SD-2.1 UNet, ldm/modules/diffusionmodules/openaimodel.py; its first-level
SpatialTransformers attend over L = 128^2 = 16384 tokens, d = 64, ldm/modules/attention.py:171-203),
as the relay DDIM calls it (model/ddim_sampler_relay.py:180-231, apply_model -> eps), at t = 151,
with the synthetic weights (rdeic_amd/weights.py via the CPU twin oracle/weights.c).

Inputs, regenerated bit for bit on the device by the GPU test:
  x          [1, 4, 128, 128]   counter-based uniform (rdeic_fill_uniform, X_SEED, [-X_SCALE, X_SCALE))
  guide_hint [1, 256, 128, 128] counter-based uniform (HINT_SEED, [-HINT_SCALE, HINT_SCALE))
  context    [1, 77, 1024]      rdeic_amd.synthetic.synth_context() (seeded torch CPU generator)
Both are generated in NHWC (the device layout) and permuted to NCHW for the reference.
Stored: the whole eps [128, 128, 4] fp32 (256 KB) in NHWC.

Run in the development container only (the reference does not exist on the GPU box):
    python -m tests.golden.make_eps1024_golden
Output (committed): tests/golden/eps_1024.npz."""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import weights_cpu  # noqa: E402
from rdeic_amd.config import CONFIG  # noqa: E402
from rdeic_amd.synthetic import synth_context  # noqa: E402
from tests.golden import refload  # noqa: E402
from tests.golden.make_golden import fill_module  # noqa: E402

LAT, T = 128, 151
X_SEED, X_SCALE = 0xE95_1024, 1.7
HINT_SEED, HINT_SCALE = 0x41E7_1024, 1.0


def field(n_ch, seed, scale):
    a = weights_cpu.fill_uniform(n_ch * LAT * LAT, seed, scale, 0.0)
    return torch.from_numpy(a).view(1, LAT, LAT, n_ch).permute(0, 3, 1, 2).contiguous()


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    R = refload.load()
    unet = R.UNetModel(**CONFIG["unet"]).eval()
    ne = R.NoiseEstimator(**CONFIG["control"]).eval()
    fill_module(unet, "model.diffusion_model.")
    fill_module(ne, "control_model.")
    x = field(4, X_SEED, X_SCALE)
    hint = field(256, HINT_SEED, HINT_SCALE)
    ctx = synth_context()
    t0 = time.time()
    with torch.no_grad():
        e = ne(x=x, guide_hint=hint, timesteps=torch.full((1,), T, dtype=torch.long), context=ctx, base_model=unet)
    print(f"eps {time.time() - t0:.1f}s, out {tuple(e.shape)} range [{e.min().item():.3f}, {e.max().item():.3f}] "
          f"std {e.std().item():.4f}")
    np.savez_compressed(os.path.join(HERE, "eps_1024.npz"), x_seed=np.uint64(X_SEED), x_scale=np.float64(X_SCALE),
                        hint_seed=np.uint64(HINT_SEED), hint_scale=np.float64(HINT_SCALE), t=np.int64(T),
                        eps=e[0].permute(1, 2, 0).contiguous().numpy())


if __name__ == "__main__":
    main()
