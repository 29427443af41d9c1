"""Relay DDIM sampler (model/ddim_sampler_relay.py) on the HIP path.

Schedule (make_schedule :23-52, util.py:53-81): ddpm_num_timesteps = model.used_timesteps (300),
uniform DDIM timesteps range(0, 300, 300 // S) + 1, a_t = abar[tau], a_prev = [abar[0]] +
abar[tau[:-1]], sigma = eta * ... (eta = 0). The relay quirk is kept: x_T is noised at t = 299
by the caller while the first DDIM step evaluates the model at tau[-1] (151 for S = 2).
Per step (p_sample_ddim :180-231): e = apply_model(x, t); pred_x0 = (x - sqrt(1-a_t) e) / sqrt(a_t);
x' = sqrt(a_prev) pred_x0 + sqrt(1 - a_prev - sigma^2) e (+ sigma * noise, = 0 at eta = 0) —
one fused kernel with the fp32 scalars computed on the host exactly as the reference does.
The reference draws an unused `noise_like` randn per step; at eta = 0 it does not affect the
result, so no device RNG is consumed here.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ops


def make_ddim_timesteps(num_ddim_timesteps: int, num_ddpm_timesteps: int) -> np.ndarray:
    c = num_ddpm_timesteps // num_ddim_timesteps
    return np.asarray(list(range(0, num_ddpm_timesteps, c))) + 1


class DDIMSampler:
    def __init__(self, model, schedule: str = "linear", **kwargs):
        self.model = model
        self.ddpm_num_timesteps = model.used_timesteps
        self.schedule = schedule

    def make_schedule(self, ddim_num_steps: int, ddim_discretize: str = "uniform", ddim_eta: float = 0.0,
                      verbose: bool = False):
        if ddim_discretize != "uniform":
            raise NotImplementedError(ddim_discretize)
        self.ddim_timesteps = make_ddim_timesteps(ddim_num_steps, self.ddpm_num_timesteps)
        ac = self.model._sched_cpu["alphas_cumprod"]           # fp32 buffer
        self.ddim_alphas = ac[self.ddim_timesteps].numpy()     # fp32
        self.ddim_alphas_prev = np.asarray([ac[0].item()] + ac[self.ddim_timesteps[:-1]].tolist())
        self.ddim_sigmas = ddim_eta * np.sqrt((1 - self.ddim_alphas_prev) / (1 - self.ddim_alphas) *
                                              (1 - self.ddim_alphas / self.ddim_alphas_prev))
        self.ddim_sqrt_one_minus_alphas = np.sqrt(np.float32(1.0) - self.ddim_alphas)
        self.eta = ddim_eta

    def _step_scalars(self, index: int):
        f32 = np.float32
        a_t = f32(self.ddim_alphas[index])
        a_prev = f32(self.ddim_alphas_prev[index])
        sigma = f32(self.ddim_sigmas[index])
        c_sq1m = f32(self.ddim_sqrt_one_minus_alphas[index])
        c_sqa = np.sqrt(a_t)
        c_sqap = np.sqrt(a_prev)
        c_dir = np.sqrt(f32(f32(f32(1.0) - a_prev) - f32(sigma * sigma)))
        return float(c_sq1m), float(c_sqa), float(c_sqap), float(c_dir), float(sigma)

    @torch.no_grad()
    def sample_nhwc(self, S: int, x_T: torch.Tensor, guide_hint: torch.Tensor, context: torch.Tensor,
                    eta: float = 0.0, ts_tensors=None, unconditional_guidance_scale: float = 1.0,
                    uc_hint: torch.Tensor = None, uc_context: torch.Tensor = None) -> torch.Tensor:
        """Internal path: x_T fp32 NHWC, guide_hint NHWC (compute dtype). Returns samples fp32 NHWC.
        ts_tensors: optional {timestep: int64 [B] device tensor} prepared outside a recorded plan.
        Guidance (p_sample_ddim :186-192): with an unconditional (uc_hint, uc_context) and a scale
        != 1, e = e_u + scale * (e_c - e_u) where e_u is the FULL relay model (control included)
        evaluated on the unconditional hint and context."""
        guided = (uc_hint is not None or uc_context is not None) and unconditional_guidance_scale != 1.0
        self.make_schedule(S, ddim_eta=eta)
        if eta != 0.0:
            raise NotImplementedError("relay decoding uses eta = 0 (inference.py:78)")
        x = x_T.contiguous()
        B = x.shape[0]
        ts_all = np.flip(self.ddim_timesteps)
        total = len(ts_all)
        for i, step in enumerate(ts_all):
            index = total - i - 1
            ts = (ts_tensors[int(step)] if ts_tensors is not None else
                  torch.full((B,), int(step), dtype=torch.long, device=x.device))
            e = self.model.eps_nhwc(x, ts, guide_hint, context)
            if guided:
                e_u = self.model.eps_nhwc(x, ts, uc_hint, uc_context)
                e = ops.cfg_combine(e, e_u, unconditional_guidance_scale)
            c_sq1m, c_sqa, c_sqap, c_dir, _ = self._step_scalars(index)
            xp = torch.empty_like(x)
            ops.call("rdeic_ddim_step", x.data_ptr(), e.data_ptr(), x.numel(), c_sq1m, c_sqa, c_sqap, c_dir,
                     xp.data_ptr(), None, ops.stream_ptr())
            x = xp
        return x

    @torch.no_grad()
    def sample(self, S, batch_size, shape, conditioning=None, callback=None, eta=0.0, x_T=None, verbose=True,
               unconditional_guidance_scale=1.0, unconditional_conditioning=None, **kwargs):
        """Reference signature (ddim_sampler_relay.py:54-120); NCHW in / out."""
        C, H, W_ = shape
        dev = self.model.device
        if x_T is None:
            x_T = torch.randn((batch_size, C, H, W_), device=dev)
        x = ops.nchw_to_nhwc(x_T.float().to(dev), torch.float32)
        hint = ops.nchw_to_nhwc(conditioning["guide_hint"].float().to(dev), self.model.compute_dtype)
        ctx = torch.cat(conditioning["c_crossattn"], 1)
        uc_hint = uc_ctx = None
        if unconditional_conditioning is not None and unconditional_guidance_scale != 1.0:
            uc = unconditional_conditioning
            uc_hint = ops.nchw_to_nhwc(uc["guide_hint"].float().to(dev), self.model.compute_dtype)
            uc_ctx = torch.cat(uc["c_crossattn"], 1)
        samples = self.sample_nhwc(S, x, hint, ctx, eta=eta, unconditional_guidance_scale=unconditional_guidance_scale,
                                   uc_hint=uc_hint, uc_context=uc_ctx)
        out = ops.nhwc_to_nchw(samples)
        return out, {"x_inter": [x_T, out], "pred_x0": [x_T]}
