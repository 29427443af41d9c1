"""RDEIC codec model — the reference's model/rdeic.py API surface on the MI355X path.

API parity (model/rdeic.py, ldm/models/diffusion/ddpm.py):
  apply_condition_compress(x, stream_path, H, W) -> bpp          rdeic.py:659-669
  apply_condition_decompress(stream_path) -> (c_latent, guide_hint) rdeic.py:671-676
  q_sample(x_start, t, noise)                                      ddpm.py:357-360
  apply_model(x_noisy, t, cond) -> eps                             rdeic.py:688-698
  decode_first_stage(z)                                            ddpm.py:835-844
  alphas_cumprod & co. (register_schedule, ddpm.py:139-193), used_timesteps, parameterization,
  scale_factor, device, preprocess_model.update(force=True), load_state_dict(state_dict).
Tensors crossing this API are the reference's NCHW fp32; internally everything is NHWC and the
batched fast path (`codec_images`) never converts layouts between stages.
Text conditioning (OpenCLIP, out of scope) is supplied as a context tensor [1 or B, 77, 1024].
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import bitstream, ops
from .compression import Compression
from .config import default_config
from .params import ParamStore
from .unet import NoiseEstimator
from .vae import AutoencoderKL


def make_schedule(timesteps: int, linear_start: float, linear_end: float) -> Dict[str, torch.Tensor]:
    """register_schedule('linear') buffers: fp64 numpy math, stored fp32 (ddpm.py:139-193, util.py:21-50)."""
    betas = (torch.linspace(linear_start ** 0.5, linear_end ** 0.5, timesteps, dtype=torch.float64) ** 2).numpy()
    alphas = 1.0 - betas
    ac = np.cumprod(alphas, axis=0)
    ac_prev = np.append(1.0, ac[:-1])
    f = lambda a: torch.tensor(a, dtype=torch.float32)  # noqa: E731
    return dict(betas=f(betas), alphas_cumprod=f(ac), alphas_cumprod_prev=f(ac_prev),
                sqrt_alphas_cumprod=f(np.sqrt(ac)), sqrt_one_minus_alphas_cumprod=f(np.sqrt(1.0 - ac)),
                log_one_minus_alphas_cumprod=f(np.log(1.0 - ac)), sqrt_recip_alphas_cumprod=f(np.sqrt(1.0 / ac)),
                sqrt_recipm1_alphas_cumprod=f(np.sqrt(1.0 / ac - 1)),
                posterior_variance=f(betas * (1.0 - ac_prev) / (1.0 - ac)),
                posterior_log_variance_clipped=f(np.log(np.maximum(betas * (1.0 - ac_prev) / (1.0 - ac), 1e-20))),
                posterior_mean_coef1=f(betas * np.sqrt(ac_prev) / (1.0 - ac)),
                posterior_mean_coef2=f((1.0 - ac_prev) * np.sqrt(alphas) / (1.0 - ac)))


class RDEIC:
    parameterization = "eps"

    def __init__(self, config: Optional[dict] = None, compute_dtype=torch.bfloat16, device="cuda"):
        cfg = config or default_config()
        self.cfg = cfg
        self.store = ParamStore(compute_dtype, device)
        self.control_model = NoiseEstimator(self.store, cfg["unet"], cfg["control"])
        self.first_stage_model = AutoencoderKL(self.store, cfg["ddconfig"], cfg["embed_dim"])
        self.preprocess_model = Compression(self.store, **cfg["compression"])
        self.scale_factor = float(cfg["scale_factor"])
        self.num_timesteps = int(cfg["timesteps"])
        self.used_timesteps = int(cfg["used_timesteps"])
        self.linear_start, self.linear_end = float(cfg["linear_start"]), float(cfg["linear_end"])
        self.channels = 4
        sched = make_schedule(self.num_timesteps, cfg["linear_start"], cfg["linear_end"])
        self._sched_cpu = sched
        self.device = torch.device(device)
        for k, v in sched.items():
            setattr(self, k, v.to(self.device))
        from .plan import PlanCache
        self.use_plans = True
        self._plans = PlanCache()
        self._consts = {}

    # ------------------------------------------------------------------ weights
    @property
    def compute_dtype(self):
        return self.store.compute_dtype

    def init_synthetic(self, seed: Optional[int] = None, rate_gain: float = 1.0):
        """Synthetic weights (rdeic_amd/weights.py); rate_gain is the bpp knob (weights.RATE_LAYERS)."""
        from . import weights as W
        self.store.init_synthetic(W.GLOBAL_SEED if seed is None else seed, rate_gain)
        self._clear_plans()  # recorded plans point at the previous packed weights
        return self

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        """Load reference-named weights (e.g. a RDEIC checkpoint's state_dict). Non-parameter buffers of the
        reference (schedules, entropy tables, scale_list, cond_stage_model) are ignored."""
        self.store.load_state_dict({k: v for k, v in sd.items() if k in self.store.shapes}, strict=strict)
        self._clear_plans()
        return self

    @property
    def use_plans(self) -> bool:
        return self._use_plans

    @use_plans.setter
    def use_plans(self, v: bool):
        """Launch-plan replay for every fixed-shape region (compress, decompress, relay + decode)."""
        self._use_plans = bool(v)
        self.preprocess_model.use_plans = bool(v)

    def session(self) -> "RDEIC":
        """A codec session sharing this model's weights, tables and kernels but with its own launch
        plans, pinned buffers and per-call host state: one session per host thread / HIP stream lets
        two batches be in flight at once (one batch's host entropy coding overlaps the other's GPU
        work). Record each session's plans (run it once) before running sessions concurrently."""
        import copy
        from .plan import PlanCache
        s = copy.copy(self)
        s._plans = PlanCache()
        s._consts = {}
        pm = copy.copy(self.preprocess_model)
        pm._plans = PlanCache()
        pm._io = {}
        pm.__dict__.pop("_pin_cache", None)
        s.preprocess_model = pm
        return s

    def _clear_plans(self):
        self._plans.clear()
        self.preprocess_model._plans.clear()
        self.preprocess_model._en = None

    def param_shapes(self):
        return dict(self.store.shapes)

    # ------------------------------------------------------------------ internal NHWC stages
    def encode_images_nhwc(self, img_u8: torch.Tensor) -> torch.Tensor:
        """uint8 [B,H,W,3] (device) -> h = 0.18215 * Encoder.forward_hc(x*2-1), NHWC compute dtype."""
        B, H, W_, _ = img_u8.shape
        # bf16: 8 channels (3 + 5 zeros) so the VAE's conv_in gathers 16-byte vectors (cin-padded weights)
        cpad = 8 if self.compute_dtype == torch.bfloat16 else 3
        x = torch.empty((B, H, W_, cpad), dtype=self.compute_dtype, device=img_u8.device)
        ops.call("rdeic_image_u8_to_nhwc", img_u8.contiguous().data_ptr(), B, H, W_, x.data_ptr(), cpad,
                 ops.dt_code(x), ops.stream_ptr())
        return self.first_stage_model.encode_hc(x, out_mul=self.scale_factor)

    def encode_nchw_nhwc(self, x: torch.Tensor) -> torch.Tensor:
        """x in [0,1] NCHW fp32 -> h (apply_condition_compress's x*2-1 fused into the layout conversion)."""
        xh = ops.nchw_to_nhwc(x.to(self.device), self.compute_dtype, mul=2.0, add=-1.0)
        return self.first_stage_model.encode_hc(xh, out_mul=self.scale_factor)

    def q_sample_nhwc(self, x0: torch.Tensor, t: torch.Tensor, noise: torch.Tensor) -> torch.Tensor:
        B = x0.shape[0]
        t = t.to(self.device).long()
        a = self.sqrt_alphas_cumprod[t].contiguous()
        b = self.sqrt_one_minus_alphas_cumprod[t].contiguous()
        out = torch.empty_like(x0)
        ops.call("rdeic_axpby", x0.contiguous().data_ptr(), noise.contiguous().data_ptr(), B, x0[0].numel(),
                 a.data_ptr(), b.data_ptr(), out.data_ptr(), ops.stream_ptr())
        return out

    def eps_nhwc(self, x: torch.Tensor, t: torch.Tensor, guide_hint: torch.Tensor, context: torch.Tensor):
        return self.control_model.forward(x, guide_hint, t, context.to(self.device))

    def eps_uncond_nhwc(self, x: torch.Tensor, t: torch.Tensor, context: torch.Tensor):
        """Base UNet alone, no control branch (NoiseEstimator.forward_unconditional, rdeic.py:214-235)."""
        return self.control_model.forward_unconditional(x, t, context.to(self.device))

    def decode_nhwc(self, z: torch.Tensor, out_f32: bool = True, consts=None) -> torch.Tensor:
        """z: fp32 NHWC latent sample -> decoder output NHWC [B,8h,8w,3] (1/scale_factor fused)."""
        B = z.shape[0]
        zs = torch.empty_like(z)
        consts = consts or self._region_consts(B, 0, z.device)
        inv, zero = consts["inv_scale"], consts["zero"]
        ops.call("rdeic_axpby", z.contiguous().data_ptr(), z.contiguous().data_ptr(), B, z[0].numel(), inv.data_ptr(),
                 zero.data_ptr(), zs.data_ptr(), ops.stream_ptr())
        zc = ops.cast(zs, self.compute_dtype)
        return self.first_stage_model.decode(zc, out_f32=out_f32)

    def to_image_u8(self, x: torch.Tensor) -> torch.Tensor:
        B, H, W_, C = x.shape
        img = torch.empty((B, H, W_, 3), dtype=torch.uint8, device=x.device)
        ops.call("rdeic_nhwc_to_image_u8", x.data_ptr(), B, H, W_, ops.pix_ld(x), img.data_ptr(), ops.dt_code(x),
                 ops.stream_ptr())
        return img

    # ------------------------------------------------------------------ reference API
    @torch.no_grad()
    def apply_condition_compress(self, x: torch.Tensor, stream_path: str, H: int, W: int) -> float:
        """x: [1,3,H,W] in [0,1]. Writes the bitstream file, returns bpp = 8*filesize/(H*W)."""
        if x.shape[0] != 1:
            raise ValueError("apply_condition_compress codes one image per file (the reference's decompress "
                             "supports batch 1 only); use compress_images for batches")
        h = self.encode_nchw_nhwc(x)
        out = self.preprocess_model.compress(h)[0]
        with Path(stream_path).open("wb") as f:
            bitstream.write_body(f, out["shape"], out["strings"])
        size = bitstream.filesize(stream_path)
        return float(size) * 8 / (H * W)

    @torch.no_grad()
    def apply_condition_decompress(self, stream_path: str):
        with Path(stream_path).open("rb") as f:
            strings, shape = bitstream.read_body(f)
        c_lat, hint = self.preprocess_model.decompress([strings], shape, device=self.device)
        return ops.nhwc_to_nchw(c_lat), ops.nhwc_to_nchw(hint)

    def q_sample(self, x_start: torch.Tensor, t: torch.Tensor, noise: Optional[torch.Tensor] = None):
        if noise is None:
            noise = torch.randn_like(x_start)
        B, C, H, W_ = x_start.shape
        out = self.q_sample_nhwc(x_start.float().contiguous(), t, noise.float().contiguous().to(x_start.device))
        return out  # elementwise: layout-agnostic, returned in the caller's (NCHW) layout

    @torch.no_grad()
    def apply_model(self, x_noisy: torch.Tensor, t: torch.Tensor, cond: dict) -> torch.Tensor:
        ctx = torch.cat(cond["c_crossattn"], 1)
        x = ops.nchw_to_nhwc(x_noisy.float().to(self.device), torch.float32)
        hint = cond["guide_hint"]
        hint_nhwc = ops.nchw_to_nhwc(hint.float().to(self.device), self.compute_dtype)
        eps = self.eps_nhwc(x, t.to(self.device), hint_nhwc, ctx)
        return ops.nhwc_to_nchw(eps)

    @torch.no_grad()
    def apply_model_unconditional(self, x_noisy: torch.Tensor, t: torch.Tensor, cond: dict) -> torch.Tensor:
        """rdeic.py:700-709: the base UNet with cond's text context, no control features."""
        ctx = torch.cat(cond["c_crossattn"], 1)
        x = ops.nchw_to_nhwc(x_noisy.float().to(self.device), torch.float32)
        return ops.nhwc_to_nchw(self.eps_uncond_nhwc(x, t.to(self.device), ctx))

    @torch.no_grad()
    def decode_first_stage(self, z: torch.Tensor) -> torch.Tensor:
        zn = ops.nchw_to_nhwc(z.float().to(self.device), torch.float32)
        return ops.nhwc_to_nchw(self.decode_nhwc(zn, out_f32=True))

    # ------------------------------------------------------------------ batched codec fast path
    @torch.no_grad()
    def compress_images(self, img_u8: torch.Tensor) -> List[bytes]:
        """uint8 [B,H,W,3] (H, W multiples of 64) -> B bitstream bodies (reference file format)."""
        img = img_u8.to(self.device).contiguous()
        outs = self.preprocess_model.compress_with(self.encode_images_nhwc, img)  # VAE encoder in the same plan
        return [bitstream.pack_body(o["shape"], o["strings"]) for o in outs]

    @torch.no_grad()
    def decompress_bodies(self, bodies: Sequence[bytes]):
        parsed = [bitstream.unpack_body(b) for b in bodies]
        shape = parsed[0][1]
        if any(p[1] != shape for p in parsed):
            raise ValueError("batched decompress needs one latent shape per batch")
        return self.preprocess_model.decompress([p[0] for p in parsed], shape, device=self.device)

    @staticmethod
    def _sampler(model, sampler: str):
        if sampler == "ddim":
            from .ddim_sampler_relay import DDIMSampler
            return DDIMSampler(model)
        if sampler == "ddpm":
            from .spaced_sampler_relay import SpacedSampler
            return SpacedSampler(model, var_type="fixed_small")  # inference.py:47-48
        raise ValueError(f"sampler {sampler!r} (ddpm | ddim)")

    def _step_timesteps(self, steps: int, sampler: str):
        if sampler == "ddpm":
            from .spaced_sampler_relay import space_timesteps
            return sorted(space_timesteps(self.used_timesteps, str(steps)))
        from .ddim_sampler_relay import make_ddim_timesteps
        return [int(t) for t in make_ddim_timesteps(steps, self.used_timesteps)]

    @torch.no_grad()
    def relay_sample_nhwc(self, c_latent: torch.Tensor, guide_hint: torch.Tensor, context: torch.Tensor,
                          noise: torch.Tensor, steps: int, sampler: str = "ddim", step_noise=None) -> torch.Tensor:
        """x_T = q_sample(c_latent, used_timesteps-1, noise); relay DDIM (eta=0) or spaced DDPM sampling."""
        B = c_latent.shape[0]
        t = torch.full((B,), self.used_timesteps - 1, dtype=torch.long, device=self.device)
        x = self.q_sample_nhwc(c_latent, t, noise)
        if sampler == "ddpm":
            return self._sampler(self, sampler).sample_nhwc(steps, x, guide_hint, context, step_noise=step_noise)
        return self._sampler(self, sampler).sample_nhwc(steps, x, guide_hint, context)

    def _region_consts(self, B: int, steps: int, device, sampler: str = "ddim") -> dict:
        """Per-(batch, steps, sampler) device constants of the relay + decode region, made outside
        any recorded launch plan (a plan replays only librdeic_hip launches)."""
        key = (B, steps, str(device), sampler)
        c = self._consts.get(key)
        if c is None:
            t = torch.full((B,), self.used_timesteps - 1, dtype=torch.long, device=device)
            c = {"qa": self.sqrt_alphas_cumprod[t].contiguous(), "qb": self.sqrt_one_minus_alphas_cumprod[t].contiguous(),
                 "inv_scale": torch.full((B,), 1.0 / self.scale_factor, dtype=torch.float32, device=device),
                 "zero": torch.zeros((B,), dtype=torch.float32, device=device), "ts": {}}
            if steps:
                for st in self._step_timesteps(steps, sampler):
                    c["ts"][int(st)] = torch.full((B,), int(st), dtype=torch.long, device=device)
            self._consts[key] = c
        return c

    def _relay_decode_u8(self, c_latent, guide_hint, context, noise, steps: int, sampler: str = "ddim",
                         step_noise=None):
        """q_sample(c_latent, 299, noise) -> relay sampler -> VAE decode -> uint8 NHWC (launches only).
        step_noise: [steps, B, h, w, 4] fp32 (ddpm only)."""
        B = c_latent.shape[0]
        c = self._region_consts(B, steps, c_latent.device, sampler)
        x = torch.empty_like(c_latent)
        ops.call("rdeic_axpby", c_latent.data_ptr(), noise.data_ptr(), B, c_latent[0].numel(), c["qa"].data_ptr(),
                 c["qb"].data_ptr(), x.data_ptr(), ops.stream_ptr())
        smp = self._sampler(self, sampler)
        if sampler == "ddpm":
            z = smp.sample_nhwc(steps, x, guide_hint, context, step_noise=list(step_noise.unbind(0)),
                                ts_tensors=c["ts"])
        else:
            z = smp.sample_nhwc(steps, x, guide_hint, context, ts_tensors=c["ts"])
        return self.to_image_u8(self.decode_nhwc(z, out_f32=True, consts=c))

    @torch.no_grad()
    def relay_decode_u8(self, c_latent: torch.Tensor, guide_hint: torch.Tensor, context: torch.Tensor,
                        noise: torch.Tensor, steps: int, sampler: str = "ddim", step_noise=None) -> torch.Tensor:
        """Relay denoise + VAE decode of a batch to uint8 [B,H,W,3]. With use_plans (default) the
        fixed-shape launch sequence is recorded once per shape and replayed (rdeic_amd/plan.py);
        the result is bit-identical to the eager path. sampler "ddpm" (the reference CLI default)
        needs step_noise [steps, B, h, w, 4] fp32 NHWC (the per-step randn_like draws)."""
        ctx = context.to(device=self.device, dtype=self.compute_dtype).contiguous()
        ins = [c_latent.contiguous(), guide_hint.contiguous(), ctx, noise.contiguous()]
        if sampler == "ddpm":
            if step_noise is None or tuple(step_noise.shape) != (steps,) + tuple(noise.shape):
                raise ValueError("sampler 'ddpm' needs step_noise of shape [steps, *noise.shape]")
            ins.append(step_noise.to(device=self.device, dtype=torch.float32).contiguous())
        elif sampler != "ddim":
            raise ValueError(f"sampler {sampler!r} (ddpm | ddim)")
        fn = (lambda a, b, c, d, *e: self._relay_decode_u8(a, b, c, d, steps, sampler, e[0] if e else None))
        if not self.use_plans:
            return fn(*ins)
        key = ("relay_decode", steps, sampler) + tuple((tuple(t.shape), t.dtype) for t in ins)
        return self._plans.run(key, fn, ins).clone()

    @torch.no_grad()
    def codec_images(self, img_u8: torch.Tensor, context: torch.Tensor, noise_nchw: torch.Tensor, steps: int = 2,
                     sampler: str = "ddim", step_noise_nchw: Optional[torch.Tensor] = None):
        """The full hot path on a batch: compress -> bytes -> decompress -> relay denoise -> VAE decode -> u8.
        step_noise_nchw: [steps, B, 4, h, w] (sampler "ddpm"). Returns (uint8 [B,H,W,3] on device, bodies)."""
        bodies = self.compress_images(img_u8)
        c_lat, hint = self.decompress_bodies(bodies)
        noise = ops.nchw_to_nhwc(noise_nchw.float().to(self.device), torch.float32)
        step_noise = None
        if step_noise_nchw is not None:
            step_noise = torch.stack([ops.nchw_to_nhwc(n.float().to(self.device), torch.float32)
                                      for n in step_noise_nchw])
        return self.relay_decode_u8(c_lat, hint, context, noise, steps, sampler, step_noise), bodies
