"""Golden vectors for classifier-free guidance in both relay samplers, from the reference's own
DDIMSampler (model/ddim_sampler_relay.py:180-231) and SpacedSampler (model/spaced_sampler_relay.py:
172-191, predict_noise :277-283) run in this container. Output: tests/golden/cfg_sampler.npz.

The eps networks are fixed affine stand-ins, so the fixture pins the samplers' guidance arithmetic
and their branch semantics, not the network (e2e_128.npz pins that):
  * DDIM  apply_model(x, t, c)                = 0.25 x + W[t] + 0.5 c["guide_hint"]
    (the unconditional pass is apply_model on the unconditional dict — control included);
  * spaced apply_model(x, t, c)               = 0.25 x + W[t]
           apply_model_unconditional(x, t, c) = -0.1 x + U[t]   (base UNet stand-in, same c).
W[t] / U[t] are seeded per timestep (1000 + t / 2000 + t). Spaced step noise is recorded by
patching torch.randn_like.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_cfg_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden import refload  # noqa: E402

SHAPE = (2, 4, 8, 8)
# (steps, scale, with_uncond, seed)
DDIM_CASES = [(2, 3.0, True, 21), (5, 7.5, True, 22), (2, 3.0, False, 23)]
# (steps, scale, with_uncond, var_type, seed)
SPACED_CASES = [(2, 3.0, False, "fixed_small", 31), (5, 1.0, True, "fixed_small", 32), (3, 4.5, False, "fixed_large", 33)]


def w_cond(t: int) -> torch.Tensor:
    return torch.randn(SHAPE, generator=torch.Generator().manual_seed(1000 + t))


def w_uncond(t: int) -> torch.Tensor:
    return torch.randn(SHAPE, generator=torch.Generator().manual_seed(2000 + t))


class StandIn:
    """The attributes the samplers read from RDEIC (ddpm.py register_schedule and config)."""
    num_timesteps = 1000
    used_timesteps = 300
    linear_start = 0.00085
    linear_end = 0.0120
    parameterization = "eps"
    device = torch.device("cpu")

    def __init__(self):
        betas = (torch.linspace(0.00085 ** 0.5, 0.0120 ** 0.5, 1000, dtype=torch.float64) ** 2).numpy()
        ac = np.cumprod(1.0 - betas, axis=0)
        self.betas = torch.tensor(betas, dtype=torch.float32)
        self.alphas_cumprod = torch.tensor(ac, dtype=torch.float32)
        self.alphas_cumprod_prev = torch.tensor(np.append(1.0, ac[:-1]), dtype=torch.float32)
        self.calls = []

    def apply_model(self, x, t, c):
        self.calls.append(("c", int(t[0])))
        e = x * 0.25 + w_cond(int(t[0]))
        if c is not None and "guide_hint" in c:
            e = e + c["guide_hint"] * 0.5
        return e

    def apply_model_unconditional(self, x, t, c):
        self.calls.append(("u", int(t[0])))
        return x * -0.1 + w_uncond(int(t[0]))


def main():
    R = refload.load()
    out = {}
    R.DDIMSampler.register_buffer = lambda self, name, attr: setattr(self, name, attr)  # skip .to("cuda")
    for k, (steps, scale, with_uc, seed) in enumerate(DDIM_CASES):
        g = torch.Generator().manual_seed(seed)
        x_T = torch.randn(SHAPE, generator=g)
        hint = torch.randn(SHAPE, generator=g)
        uc_hint = torch.randn(SHAPE, generator=g)
        m = StandIn()
        smp = R.DDIMSampler(m)
        cond = {"guide_hint": hint}
        uc = {"guide_hint": uc_hint} if with_uc else None
        samples, _ = smp.sample(S=steps, batch_size=SHAPE[0], shape=SHAPE[1:], conditioning=cond,
                                unconditional_conditioning=uc, unconditional_guidance_scale=scale,
                                x_T=x_T.clone(), eta=0, verbose=False)
        pre = f"ddim{k}_"
        out[pre + "steps"] = np.int64(steps)
        out[pre + "scale"] = np.float64(scale)
        out[pre + "with_uc"] = np.int64(with_uc)
        out[pre + "x_T"] = x_T.numpy()
        out[pre + "hint"] = hint.numpy()
        out[pre + "uc_hint"] = uc_hint.numpy()
        out[pre + "samples"] = samples.numpy()
        print(f"ddim {k}: S={steps} scale={scale} uc={with_uc} calls={m.calls}")
    for k, (steps, scale, with_uc, var, seed) in enumerate(SPACED_CASES):
        g = torch.Generator().manual_seed(seed)
        x_T = torch.randn(SHAPE, generator=g)
        noises = [torch.randn(SHAPE, generator=g) for _ in range(steps)]
        m = StandIn()
        smp = R.SpacedSampler(m, var_type=var)
        it = iter(noises)
        orig = torch.randn_like
        torch.randn_like = lambda x, *a, **kw: next(it).to(x.dtype)
        try:
            samples = smp.sample(steps, SHAPE, conditioning={}, x_T=x_T.clone(), unconditional_guidance_scale=scale,
                                 unconditional_conditioning={} if with_uc else None)
        finally:
            torch.randn_like = orig
        pre = f"spaced{k}_"
        out[pre + "steps"] = np.int64(steps)
        out[pre + "scale"] = np.float64(scale)
        out[pre + "with_uc"] = np.int64(with_uc)
        out[pre + "var"] = np.frombuffer(var.encode(), dtype=np.uint8)
        out[pre + "x_T"] = x_T.numpy()
        out[pre + "noise"] = np.stack([n.numpy() for n in noises])
        out[pre + "samples"] = samples.numpy()
        print(f"spaced {k}: S={steps} scale={scale} uc={with_uc} {var} calls={m.calls}")
    path = os.path.join(HERE, "cfg_sampler.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
