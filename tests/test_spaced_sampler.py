"""Relay spaced (DDPM) sampler: schedule, timestep spacing and the sampled latents against the
reference's own SpacedSampler (tests/golden/make_spaced_golden.py -> spaced_sampler.npz, with a
fixed affine stand-in for the eps network and recorded step noise)."""
import os

import numpy as np
import pytest
import torch

GOLD = os.path.join(os.path.dirname(__file__), "golden", "spaced_sampler.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def _cases(g, prefix):
    return sorted({k.split("_")[0] for k in g.files if k.startswith(prefix)})


def stand_in_w(t: int, shape) -> torch.Tensor:  # make_spaced_golden.stand_in_w
    return torch.randn(shape, generator=torch.Generator().manual_seed(1000 + t))


class StandIn:
    num_timesteps = 1000
    used_timesteps = 300
    linear_start = 0.00085
    linear_end = 0.0120


def test_space_timesteps_match_reference(g):
    from oracle import model_ref as M
    from rdeic_amd.spaced_sampler_relay import space_timesteps
    for c in _cases(g, "spec"):
        n, spec = int(g[c + "_n"]), g[c + "_spec"].tobytes().decode()
        want = g[c + "_steps"].tolist()
        assert sorted(space_timesteps(n, spec)) == want, spec
        assert sorted(M.space_timesteps(n, spec)) == want, spec
    assert sorted(space_timesteps(300, "2")) == [0, 299]
    assert sorted(space_timesteps(300, "5")) == [0, 75, 150, 224, 299]


def test_schedule_matches_reference_float64(g):
    from rdeic_amd.spaced_sampler_relay import SpacedSampler
    for c in _cases(g, "case"):
        smp = SpacedSampler(StandIn(), var_type=g[c + "_var"].tobytes().decode())
        smp.make_schedule(int(g[c + "_steps"]))
        for key in ("betas", "timesteps", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_recip_alphas_cumprod",
                    "sqrt_recipm1_alphas_cumprod", "posterior_variance", "posterior_log_variance_clipped",
                    "posterior_mean_coef1", "posterior_mean_coef2"):
            assert np.array_equal(np.asarray(getattr(smp, key)), g[c + "_" + key]), (c, key)
        assert smp.step_scalars(0)[4] == 0.0  # no noise at the last step
        assert smp.step_timesteps(int(g[c + "_steps"])) == g[c + "_eps_t"].tolist()


def test_oracle_spaced_relay_bit_exact(g):
    from oracle import model_ref as M
    for c in _cases(g, "case"):
        shape = g[c + "_x_T"].shape
        noise = [torch.from_numpy(n) for n in g[c + "_noise"]]
        out = M.spaced_relay(None, torch.from_numpy(g[c + "_x_T"]), None, None, int(g[c + "_steps"]), noise,
                             var_type=g[c + "_var"].tobytes().decode(),
                             eps_fn=lambda x, t: x * 0.25 + stand_in_w(int(t[0]), shape))
        assert np.array_equal(out.numpy(), g[c + "_samples"]), c


@pytest.mark.gpu
def test_spaced_step_kernel_bit_exact(gpu, g):
    """SpacedSampler.sample_nhwc through rdeic_spaced_step (C ABI) == the reference's samples,
    bit for bit (the stand-in eps model runs as torch ops on the GPU)."""
    from rdeic_amd import ops
    from rdeic_amd.spaced_sampler_relay import SpacedSampler

    class Mock(StandIn):
        def __init__(self, shape):
            self.shape = shape

        def eps_nhwc(self, x, ts, hint, ctx):
            w = ops.nchw_to_nhwc(stand_in_w(int(ts[0]), self.shape).cuda(), torch.float32)
            return x * 0.25 + w

    for c in _cases(g, "case"):
        shape = g[c + "_x_T"].shape
        x = ops.nchw_to_nhwc(torch.from_numpy(g[c + "_x_T"]).cuda(), torch.float32)
        nz = [ops.nchw_to_nhwc(torch.from_numpy(n).cuda(), torch.float32) for n in g[c + "_noise"]]
        smp = SpacedSampler(Mock(shape), var_type=g[c + "_var"].tobytes().decode())
        out = smp.sample_nhwc(int(g[c + "_steps"]), x, None, None, step_noise=nz)
        got = ops.nhwc_to_nchw(out).cpu().numpy()
        assert np.array_equal(got, g[c + "_samples"]), (c, np.abs(got - g[c + "_samples"]).max())


@pytest.mark.gpu
def test_spaced_relay_fp32_matches_oracle(gpu):
    """Full network: relay spaced sampling (q_sample at t=299, then t=299 -> 0) of the fp32 HIP
    path vs the CPU oracle on the reference's decompressed latents of golden image 0."""
    from oracle import model_ref as M
    from rdeic_amd import ops
    from rdeic_amd.rdeic import RDEIC
    e2e = np.load(os.path.join(os.path.dirname(__file__), "golden", "e2e_128.npz"))
    m = RDEIC(compute_dtype=torch.float32).init_synthetic()
    c_lat = torch.from_numpy(e2e["img0_c_latent"])
    hint = torch.from_numpy(e2e["img0_guide_hint"])
    ctx = torch.from_numpy(e2e["context"])
    gen = torch.Generator().manual_seed(231)
    noise = torch.randn(c_lat.shape, generator=gen)
    step_noise = [torch.randn(c_lat.shape, generator=gen) for _ in range(2)]
    sch = M.schedule()
    x_T = sch["sqrt_alphas_cumprod"][299] * c_lat + sch["sqrt_one_minus_alphas_cumprod"][299] * noise
    ref = M.spaced_relay(M.synthetic_state_dict(), x_T, hint, ctx, 2, step_noise)
    nhwc = lambda t: ops.nchw_to_nhwc(t.cuda(), torch.float32)  # noqa: E731
    z = m.relay_sample_nhwc(nhwc(c_lat), nhwc(hint), ctx.cuda(), nhwc(noise), 2, sampler="ddpm",
                            step_noise=[nhwc(n) for n in step_noise])
    got = ops.nhwc_to_nchw(z).cpu().numpy()
    err = np.abs(got - ref.numpy()).max() / np.abs(ref.numpy()).max()
    assert err < 1e-3, err


@pytest.mark.gpu
def test_codec_ddpm_plan_matches_eager(gpu):
    """bf16 codec with the spaced sampler: plan replay == eager, and the step noise is consumed."""
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    m.preprocess_model.update(force=True)
    S, B = 128, 2
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 900 + i) for i in range(B)])).cuda()
    ctx = synth_context().cuda()
    noise, steps_nz = relay_noise((B, 4, S // 8, S // 8), 231, 2)
    outs = []
    for plans in (False, True, True):
        m.use_plans = plans
        out, bodies = m.codec_images(imgs, ctx, noise, steps=2, sampler="ddpm", step_noise_nchw=steps_nz)
        outs.append(out)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    out2, _ = m.codec_images(imgs, ctx, noise, steps=2, sampler="ddpm", step_noise_nchw=steps_nz * 0)
    assert not torch.equal(out2, outs[0])
