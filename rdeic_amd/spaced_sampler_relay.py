"""Relay spaced (DDPM) sampler (model/spaced_sampler_relay.py) on the HIP path — the reference
CLI's default `--sampler ddpm` (inference.py:47-48,102).

The schedule is computed on the host in float64, exactly as the reference does it:
  space_timesteps(used_timesteps, str(S))                  spaced_sampler_relay.py:11-61
  make_schedule: betas re-spaced from the original 1000-step linear schedule, then the
  posterior coefficients and variances                     :88-142
Each step is p_sample_spaced (:349-384), with _predict_xstart_from_eps (:270-275) and
q_posterior_mean_variance (:154-170), and runs as one fused kernel, rdeic_spaced_step. The kernel
takes the fp32 scalars that the reference extracts with _extract_into_tensor
(`torch.from_numpy(arr)[t].float()`, :65-77):
  pred_x0 = A * x - B * e           A = sqrt_recip_alphas_cumprod[i], B = sqrt_recipm1_alphas_cumprod[i]
  mean    = C1 * pred_x0 + C2 * x   C1, C2 = posterior_mean_coef1 / 2 [i]
  x'      = mean + S * noise        S = nonzero_mask * sqrt(model_variance[i])  (0 at i = 0)
Every product and sum is rounded on its own (no fma contraction). That is the reference's eager
fp32 op order, so the update itself is bit-exact. The model is evaluated at the kept original
timesteps themselves (e.g. 299 then 0 for S = 2), as the reference does.
The reference draws each step's noise with torch.randn_like(x) on its device (:378). Here the
caller passes the noise tensors: inference.py draws them from its seeded CPU generator in the
reference order. When the caller passes none, torch.randn_like is used.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from . import ops


def space_timesteps(num_timesteps: int, section_counts) -> set:
    """The original-process timesteps to keep (guided-diffusion respace.py semantics,
    spaced_sampler_relay.py:11-61): equal sections, each strided to its count; "ddimN" = the
    DDIM paper's fixed integer stride."""
    if isinstance(section_counts, str):
        if section_counts.startswith("ddim"):
            want = int(section_counts[len("ddim"):])
            for stride in range(1, num_timesteps):
                if len(range(0, num_timesteps, stride)) == want:
                    return set(range(0, num_timesteps, stride))
            raise ValueError(f"cannot create exactly {num_timesteps} steps with an integer stride")
        section_counts = [int(x) for x in section_counts.split(",")]
    size_per, extra = divmod(num_timesteps, len(section_counts))
    start, kept = 0, []
    for i, count in enumerate(section_counts):
        size = size_per + (1 if i < extra else 0)
        if size < count:
            raise ValueError(f"cannot divide section of {size} steps into {count}")
        stride = 1 if count <= 1 else (size - 1) / (count - 1)
        cur = 0.0
        for _ in range(count):
            kept.append(start + round(cur))
            cur += stride
        start += size
    return set(kept)


def linear_betas(n: int, linear_start: float, linear_end: float) -> np.ndarray:
    """make_beta_schedule('linear') (ldm/modules/diffusionmodules/util.py:21-25,50), float64."""
    return (torch.linspace(linear_start ** 0.5, linear_end ** 0.5, n, dtype=torch.float64) ** 2).numpy()


class SpacedSampler:
    def __init__(self, model, schedule: str = "linear", var_type: str = "fixed_small"):
        if schedule != "linear":
            raise NotImplementedError(f"beta schedule {schedule!r} (the RDEIC configs use 'linear')")
        if var_type not in ("fixed_small", "fixed_large"):
            raise KeyError(var_type)
        self.model = model
        self.original_num_steps = model.num_timesteps
        self.used_num_steps = model.used_timesteps
        self.schedule = schedule
        self.var_type = var_type

    def make_schedule(self, num_steps: int) -> None:
        original_ac = np.cumprod(1.0 - linear_betas(self.original_num_steps, self.model.linear_start,
                                                    self.model.linear_end), axis=0)
        used = space_timesteps(self.used_num_steps, str(num_steps))
        betas, last = [], 1.0
        for i, ac in enumerate(original_ac):
            if i in used:  # the marginal q(x_{S_t} | x_0) is kept
                betas.append(1 - ac / last)
                last = ac
        if len(betas) != num_steps:
            raise ValueError(f"{num_steps} steps requested, {len(betas)} kept")
        betas = np.array(betas, dtype=np.float64)
        self.betas = betas
        self.timesteps = np.array(sorted(used), dtype=np.int32)
        alphas = 1.0 - betas
        self.alphas_cumprod = np.cumprod(alphas, axis=0)
        self.alphas_cumprod_prev = np.append(1.0, self.alphas_cumprod[:-1])
        self.alphas_cumprod_next = np.append(self.alphas_cumprod[1:], 0.0)
        self.sqrt_alphas_cumprod = np.sqrt(self.alphas_cumprod)
        self.sqrt_one_minus_alphas_cumprod = np.sqrt(1.0 - self.alphas_cumprod)
        self.log_one_minus_alphas_cumprod = np.log(1.0 - self.alphas_cumprod)
        self.sqrt_recip_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod)
        self.sqrt_recipm1_alphas_cumprod = np.sqrt(1.0 / self.alphas_cumprod - 1)
        self.posterior_variance = betas * (1.0 - self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_log_variance_clipped = np.log(np.append(self.posterior_variance[1], self.posterior_variance[1:]))
        self.posterior_mean_coef1 = betas * np.sqrt(self.alphas_cumprod_prev) / (1.0 - self.alphas_cumprod)
        self.posterior_mean_coef2 = (1.0 - self.alphas_cumprod_prev) * np.sqrt(alphas) / (1.0 - self.alphas_cumprod)

    def model_variance(self) -> np.ndarray:
        if self.var_type == "fixed_large":
            return np.append(self.posterior_variance[1], self.betas[1:])
        return self.posterior_variance

    def step_scalars(self, index: int):
        """(A, B, C1, C2, S) of step `index` as the reference's fp32 tensors hold them."""
        f32 = np.float32
        s = f32(0.0) if index == 0 else np.sqrt(f32(self.model_variance()[index]))
        return (float(f32(self.sqrt_recip_alphas_cumprod[index])), float(f32(self.sqrt_recipm1_alphas_cumprod[index])),
                float(f32(self.posterior_mean_coef1[index])), float(f32(self.posterior_mean_coef2[index])), float(s))

    def step_timesteps(self, num_steps: int):
        """Model timesteps in the order the steps evaluate them (high to low)."""
        return [int(t) for t in np.flip(np.array(sorted(space_timesteps(self.used_num_steps, str(num_steps)))))]

    @torch.no_grad()
    def sample_nhwc(self, steps: int, x_T: torch.Tensor, guide_hint: torch.Tensor, context: torch.Tensor,
                    step_noise: Optional[Sequence[torch.Tensor]] = None, ts_tensors=None,
                    unconditional_guidance_scale: float = 1.0, guided: bool = False) -> torch.Tensor:
        """Internal path: x_T fp32 NHWC, guide_hint NHWC (compute dtype); step_noise[i] (fp32, x's
        layout) is the noise the i-th step draws (steps taken from high t to low). Returns fp32 NHWC.
        ts_tensors: optional {timestep: int64 [B] device tensor} prepared outside a recorded plan.
        Guidance (predict_noise :277-283): when `guided` (an unconditional conditioning was given or
        the scale != 1), e = e_u + scale * (e_c - e_u) with e_u from the base UNet alone on the SAME
        text context (apply_model_unconditional, no control) — unlike the DDIM sampler."""
        guided = guided or unconditional_guidance_scale != 1.0
        self.make_schedule(steps)
        x = x_T.contiguous()
        B = x.shape[0]
        time_range = np.flip(self.timesteps)
        total = len(self.timesteps)
        if step_noise is not None and len(step_noise) < total:
            raise ValueError(f"{total} steps need {total} noise tensors, got {len(step_noise)}")
        for i, step in enumerate(time_range):
            index = total - i - 1
            ts = (ts_tensors[int(step)] if ts_tensors is not None else
                  torch.full((B,), int(step), dtype=torch.long, device=x.device))
            e = self.model.eps_nhwc(x, ts, guide_hint, context)
            if guided:
                e = ops.cfg_combine(e, self.model.eps_uncond_nhwc(x, ts, context), unconditional_guidance_scale)
            a, b, c1, c2, s = self.step_scalars(index)
            nz = step_noise[i] if step_noise is not None else torch.randn_like(x)
            if tuple(nz.shape) != tuple(x.shape) or nz.dtype != torch.float32 or not nz.is_contiguous():
                raise ValueError("step noise must be contiguous fp32 in x's shape")
            xp = torch.empty_like(x)
            ops.call("rdeic_spaced_step", x.data_ptr(), e.data_ptr(), nz.data_ptr(), x.numel(), a, b, c1, c2, s,
                     xp.data_ptr(), None, ops.stream_ptr())
            x = xp
        return x

    @torch.no_grad()
    def sample(self, steps, shape, conditioning=None, x_T=None, unconditional_guidance_scale=1.0,
               unconditional_conditioning=None, cond_fn=None, step_noise=None):
        """Reference signature (spaced_sampler_relay.py:172-191); NCHW in / out. step_noise: one
        NCHW fp32 tensor per step (the reference's per-step randn_like), or None."""
        if cond_fn is not None:
            raise NotImplementedError("classifier guidance (cond_fn) is not on the relay-decode hot path")
        dev = self.model.device
        if x_T is None:
            x_T = torch.randn(shape, device=dev)
        x = ops.nchw_to_nhwc(x_T.float().to(dev), torch.float32)
        hint = ops.nchw_to_nhwc(conditioning["guide_hint"].float().to(dev), self.model.compute_dtype)
        ctx = torch.cat(conditioning["c_crossattn"], 1)
        nz = None
        if step_noise is not None:
            nz = [ops.nchw_to_nhwc(n.float().to(dev), torch.float32) for n in step_noise]
        return ops.nhwc_to_nchw(self.sample_nhwc(steps, x, hint, ctx, step_noise=nz,
                                                 unconditional_guidance_scale=unconditional_guidance_scale,
                                                 guided=unconditional_conditioning is not None))
