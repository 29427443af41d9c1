"""Seeded synthetic inputs (no datasets / checkpoints offline):
smooth 512^2-style RGB images, the [1, 77, 1024] text context standing in for OpenCLIP(""),
and the host-side noise draws of inference.process (a discarded randn, then `noise`)."""
import numpy as np
import torch
import torch.nn.functional as F


def synth_image(h: int, w: int, seed: int) -> np.ndarray:
    """uint8 HWC: bicubic-upsampled 16x16 uniform field + 8-px checker (amp 20) + N(0, 8^2), clipped."""
    g = torch.Generator().manual_seed(int(seed))
    field = torch.rand(1, 3, 16, 16, generator=g) * 255.0
    img = F.interpolate(field, size=(h, w), mode="bicubic", align_corners=False)[0]
    yy = torch.arange(h).view(h, 1) // 8
    xx = torch.arange(w).view(1, w) // 8
    checker = (((yy + xx) % 2) * 2 - 1).float() * 20.0
    img = img + checker + torch.randn(3, h, w, generator=g) * 8.0
    return img.clamp(0, 255).round().to(torch.uint8).permute(1, 2, 0).contiguous().numpy()


def synth_context(seed: int = 1024, length: int = 77, dim: int = 1024) -> torch.Tensor:
    g = torch.Generator().manual_seed(int(seed))
    return torch.randn(1, length, dim, generator=g)


def sampler_noise(shape, seed: int):
    """(x_T_discarded, noise) in the order inference.py:64-65 draws them, from a CPU generator."""
    g = torch.Generator().manual_seed(int(seed))
    discarded = torch.randn(shape, generator=g)
    noise = torch.randn(shape, generator=g)
    return discarded, noise


def relay_noise(shape, seed: int, steps: int):
    """(noise, step_noise [steps, *shape]) from one CPU generator in the reference's draw order for
    `--sampler ddpm`: the discarded x_T randn, the q_sample noise (inference.py:64-65), then one
    randn_like per sampler step (spaced_sampler_relay.py:378)."""
    g = torch.Generator().manual_seed(int(seed))
    torch.randn(shape, generator=g)
    noise = torch.randn(shape, generator=g)
    return noise, torch.stack([torch.randn(shape, generator=g) for _ in range(steps)])


def train_draws(batch: int, h: int, w: int, slice_ch, seed: int, used_timesteps: int = 300):
    """The random draws of one adapter fine-tune step (model/rdeic.py:774-796, ddpm.py:665-672,
    compressai GaussianConditional "noise" mode), from one CPU generator in the reference's order:
    t ~ randint(0, used_timesteps) (rdeic.py:778), the posterior sample's randn
    (distributions.py:36), one U(-0.5, 0.5) per entropy slice in slice order (NCHW [B, c, h/2, w/2]
    of the 8x-down latent's y), then the p_losses randn (rdeic.py:795). h, w: latent size."""
    g = torch.Generator().manual_seed(int(seed))
    t = torch.randint(0, used_timesteps, (batch,), generator=g)
    post_eps = torch.randn((batch, 4, h, w), generator=g)
    hy, wy = h // 2, w // 2
    slice_noise = [torch.rand((batch, c, hy, wy), generator=g) - 0.5 for c in slice_ch]
    noise = torch.randn((batch, 4, h, w), generator=g)
    return dict(t=t, post_eps=post_eps, slice_noise=slice_noise, noise=noise)
