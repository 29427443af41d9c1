"""Golden vectors for the relay spaced (DDPM) sampler, from the reference's own SpacedSampler
(model/spaced_sampler_relay.py) run in this container. Output: tests/golden/spaced_sampler.npz.

Pinned: space_timesteps for several section specs, the float64 schedule of make_schedule, and
sample() for S = 2 / 5 with both variance types. The stand-in eps model is fixed and affine,
eps = 0.25 * x + W[t], with W[t] seeded per timestep. The step noise is recorded by patching
torch.randn_like. So the fixture pins the sampler's arithmetic, its timestep order and its noise
consumption. The network itself is pinned by e2e_128.npz.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_spaced_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden import refload  # noqa: E402

SHAPE = (2, 4, 8, 8)
SPEC_CASES = [(300, "2"), (300, "5"), (300, "10"), (1000, "10,15,20"), (300, "ddim50"), (100, "7,3"), (300, "1")]
SAMPLE_CASES = [(2, "fixed_small", 11), (5, "fixed_small", 12), (2, "fixed_large", 13), (3, "fixed_large", 14)]
SCHED_KEYS = ["betas", "timesteps", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_recip_alphas_cumprod",
              "sqrt_recipm1_alphas_cumprod", "posterior_variance", "posterior_log_variance_clipped",
              "posterior_mean_coef1", "posterior_mean_coef2"]


def stand_in_w(t: int) -> torch.Tensor:
    return torch.randn(SHAPE, generator=torch.Generator().manual_seed(1000 + t))


class StandIn:
    """The attributes SpacedSampler reads from RDEIC (ddpm.py config and buffers)."""
    num_timesteps = 1000
    used_timesteps = 300
    linear_start = 0.00085
    linear_end = 0.0120
    parameterization = "eps"

    def __init__(self):
        self.betas = torch.zeros(1)  # only .device is read
        self.calls = []

    def apply_model(self, x, t, c):
        self.calls.append(int(t[0]))
        return x * 0.25 + stand_in_w(int(t[0]))


def main():
    R = refload.load()
    out = {}
    for k, (n, spec) in enumerate(SPEC_CASES):
        out[f"spec{k}_n"] = np.int64(n)
        out[f"spec{k}_spec"] = np.frombuffer(spec.encode(), dtype=np.uint8)
        out[f"spec{k}_steps"] = np.array(sorted(R.space_timesteps(n, spec)), dtype=np.int64)
    for k, (steps, var, seed) in enumerate(SAMPLE_CASES):
        g = torch.Generator().manual_seed(seed)
        x_T = torch.randn(SHAPE, generator=g)
        noises = [torch.randn(SHAPE, generator=g) for _ in range(steps)]
        m = StandIn()
        smp = R.SpacedSampler(m, var_type=var)
        it = iter(noises)
        orig = torch.randn_like
        torch.randn_like = lambda x, *a, **kw: next(it).to(x.dtype)
        try:
            samples = smp.sample(steps, SHAPE, conditioning=None, x_T=x_T.clone())
        finally:
            torch.randn_like = orig
        pre = f"case{k}_"
        out[pre + "steps"] = np.int64(steps)
        out[pre + "var"] = np.frombuffer(var.encode(), dtype=np.uint8)
        out[pre + "x_T"] = x_T.numpy()
        out[pre + "noise"] = np.stack([n.numpy() for n in noises])
        out[pre + "eps_t"] = np.array(m.calls, dtype=np.int64)
        out[pre + "samples"] = samples.numpy()
        for key in SCHED_KEYS:
            out[pre + key] = np.asarray(getattr(smp, key))
        print(f"case {k}: S={steps} {var} t={m.calls} |x| {samples.abs().max():.3f}")
    path = os.path.join(HERE, "spaced_sampler.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
