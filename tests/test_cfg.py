"""Classifier-free guidance in both relay samplers against the reference's own samplers
(tests/golden/make_cfg_golden.py -> cfg_sampler.npz, affine stand-in eps networks), plus the full
network (guided relay sampling, fp32 HIP path vs the CPU oracle)."""
import os

import numpy as np
import pytest
import torch

HERE = os.path.dirname(__file__)
GOLD = os.path.join(HERE, "golden", "cfg_sampler.npz")
SHAPE = (2, 4, 8, 8)


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def _cases(g, prefix):
    return sorted({k.split("_")[0] for k in g.files if k.startswith(prefix)})


def w_cond(t: int) -> torch.Tensor:  # make_cfg_golden.w_cond
    return torch.randn(SHAPE, generator=torch.Generator().manual_seed(1000 + t))


def w_uncond(t: int) -> torch.Tensor:  # make_cfg_golden.w_uncond
    return torch.randn(SHAPE, generator=torch.Generator().manual_seed(2000 + t))


def test_golden_covers_both_branches(g):
    assert len(_cases(g, "ddim")) == 3 and len(_cases(g, "spaced")) == 3
    # DDIM without an unconditional conditioning ignores the scale (p_sample_ddim :186-187)
    assert int(g["ddim2_with_uc"]) == 0 and float(g["ddim2_scale"]) != 1.0


def test_oracle_ddim_cfg_bit_exact(g):
    from oracle import model_ref as M
    eps = lambda x, t, c: x * 0.25 + w_cond(int(t[0])) + c[0] * 0.5  # noqa: E731
    for c in _cases(g, "ddim"):
        uc = (torch.from_numpy(g[c + "_uc_hint"]), None) if int(g[c + "_with_uc"]) else None
        out = M.ddim_relay(None, torch.from_numpy(g[c + "_x_T"]), torch.from_numpy(g[c + "_hint"]), None,
                           int(g[c + "_steps"]), M.schedule(), eps_fn=eps, scale=float(g[c + "_scale"]), uc=uc)
        assert np.array_equal(out.numpy(), g[c + "_samples"]), (c, np.abs(out.numpy() - g[c + "_samples"]).max())


def test_oracle_spaced_cfg_bit_exact(g):
    from oracle import model_ref as M
    for c in _cases(g, "spaced"):
        noise = [torch.from_numpy(n) for n in g[c + "_noise"]]
        out = M.spaced_relay(None, torch.from_numpy(g[c + "_x_T"]), None, None, int(g[c + "_steps"]), noise,
                             var_type=g[c + "_var"].tobytes().decode(),
                             eps_fn=lambda x, t: x * 0.25 + w_cond(int(t[0])),
                             uncond_fn=lambda x, t: x * -0.1 + w_uncond(int(t[0])),
                             scale=float(g[c + "_scale"]), guided=bool(int(g[c + "_with_uc"])))
        assert np.array_equal(out.numpy(), g[c + "_samples"]), (c, np.abs(out.numpy() - g[c + "_samples"]).max())


class _Sched:
    num_timesteps = 1000
    used_timesteps = 300
    linear_start = 0.00085
    linear_end = 0.0120


def _mock(ops):
    from rdeic_amd.rdeic import make_schedule

    class Mock(_Sched):
        _sched_cpu = make_schedule(1000, 0.00085, 0.0120)

        def eps_nhwc(self, x, ts, hint, ctx):
            w = ops.nchw_to_nhwc(w_cond(int(ts[0])).cuda(), torch.float32)
            e = x * 0.25 + w
            return e + hint * 0.5 if hint is not None else e

        def eps_uncond_nhwc(self, x, ts, ctx):
            return x * -0.1 + ops.nchw_to_nhwc(w_uncond(int(ts[0])).cuda(), torch.float32)
    return Mock()


@pytest.mark.gpu
def test_ddim_cfg_bit_exact(gpu, g):
    """DDIMSampler.sample_nhwc with guidance (rdeic_cfg_combine + rdeic_ddim_step through the C ABI)
    == the reference's samples, bit for bit."""
    from rdeic_amd import ops
    from rdeic_amd.ddim_sampler_relay import DDIMSampler
    nhwc = lambda a: ops.nchw_to_nhwc(torch.from_numpy(a).cuda(), torch.float32)  # noqa: E731
    for c in _cases(g, "ddim"):
        smp = DDIMSampler(_mock(ops))
        smp.make_schedule(int(g[c + "_steps"]))
        # The golden ran the reference sampler on torch-CPU (register_buffer patched), whose fp32
        # sqrt is not always correctly rounded (sqrt(abar_121) is 1 ulp low). The reference's own
        # device path (CUDA, ddim_sampler_relay.py:17-21) and this build both round sqrt correctly,
        # so a case whose a_t / a_prev hit such an input is compared to a few ulp, the rest bit-exact.
        vals = np.concatenate([np.asarray(smp.ddim_alphas, np.float32), np.asarray(smp.ddim_alphas_prev, np.float32)])
        exact = np.array_equal(torch.from_numpy(vals).sqrt().numpy(), np.sqrt(vals))
        uc_hint = nhwc(g[c + "_uc_hint"]) if int(g[c + "_with_uc"]) else None
        out = smp.sample_nhwc(int(g[c + "_steps"]), nhwc(g[c + "_x_T"]), nhwc(g[c + "_hint"]), None,
                              unconditional_guidance_scale=float(g[c + "_scale"]), uc_hint=uc_hint)
        got = ops.nhwc_to_nchw(out).cpu().numpy()
        if exact:
            assert np.array_equal(got, g[c + "_samples"]), (c, np.abs(got - g[c + "_samples"]).max())
        else:
            np.testing.assert_allclose(got, g[c + "_samples"], rtol=4e-6, atol=1e-6, err_msg=c)


@pytest.mark.gpu
def test_spaced_cfg_bit_exact(gpu, g):
    from rdeic_amd import ops
    from rdeic_amd.spaced_sampler_relay import SpacedSampler
    nhwc = lambda a: ops.nchw_to_nhwc(torch.from_numpy(a).cuda(), torch.float32)  # noqa: E731
    for c in _cases(g, "spaced"):
        smp = SpacedSampler(_mock(ops), var_type=g[c + "_var"].tobytes().decode())
        out = smp.sample_nhwc(int(g[c + "_steps"]), nhwc(g[c + "_x_T"]), None, None,
                              step_noise=[nhwc(n) for n in g[c + "_noise"]],
                              unconditional_guidance_scale=float(g[c + "_scale"]),
                              guided=bool(int(g[c + "_with_uc"])))
        got = ops.nhwc_to_nchw(out).cpu().numpy()
        assert np.array_equal(got, g[c + "_samples"]), (c, np.abs(got - g[c + "_samples"]).max())


@pytest.mark.gpu
def test_guided_relay_full_network_matches_oracle(gpu):
    """Full network, fp32: guided spaced sampling (base-UNet-only uncond pass) and guided DDIM (full
    relay model on an unconditional hint/context) vs the CPU oracle on golden image 0's latents."""
    from oracle import model_ref as M
    from rdeic_amd import ops
    from rdeic_amd.ddim_sampler_relay import DDIMSampler
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.spaced_sampler_relay import SpacedSampler
    e2e = np.load(os.path.join(HERE, "golden", "e2e_128.npz"))
    m = RDEIC(compute_dtype=torch.float32).init_synthetic()
    sd = M.synthetic_state_dict()
    c_lat = torch.from_numpy(e2e["img0_c_latent"])
    hint = torch.from_numpy(e2e["img0_guide_hint"])
    ctx = torch.from_numpy(e2e["context"])
    gen = torch.Generator().manual_seed(77)
    x_T = torch.randn(c_lat.shape, generator=gen)
    step_noise = [torch.randn(c_lat.shape, generator=gen) for _ in range(2)]
    uc_hint = torch.zeros_like(hint)
    uc_ctx = torch.randn(ctx.shape, generator=gen)
    nhwc = lambda t, dt=torch.float32: ops.nchw_to_nhwc(t.cuda(), dt)  # noqa: E731

    ref = M.spaced_relay(sd, x_T, hint, ctx, 2, step_noise, scale=3.0)
    z = SpacedSampler(m).sample_nhwc(2, nhwc(x_T), nhwc(hint), ctx.cuda(), step_noise=[nhwc(n) for n in step_noise],
                                     unconditional_guidance_scale=3.0)
    got = ops.nhwc_to_nchw(z).cpu().numpy()
    err = np.abs(got - ref.numpy()).max() / np.abs(ref.numpy()).max()
    assert err < 1e-3, ("spaced", err)

    ref = M.ddim_relay(sd, x_T, hint, ctx, 2, M.schedule(), scale=2.5, uc=(uc_hint, uc_ctx))
    z = DDIMSampler(m).sample_nhwc(2, nhwc(x_T), nhwc(hint), ctx.cuda(), unconditional_guidance_scale=2.5,
                                   uc_hint=nhwc(uc_hint), uc_context=uc_ctx.cuda())
    got = ops.nhwc_to_nchw(z).cpu().numpy()
    err = np.abs(got - ref.numpy()).max() / np.abs(ref.numpy()).max()
    assert err < 1e-3, ("ddim", err)
