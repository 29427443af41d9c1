"""Launch plans (rdeic_amd/plan.py): the recorded + replayed relay/decode region is bit-identical
to the eager path, across replays with new inputs."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_relay_decode_plan_matches_eager(gpu):
    from rdeic_amd import ops
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    B, h = 2, 16
    g = torch.Generator().manual_seed(0)
    ctx = synth_context().cuda()
    outs_eager, outs_plan = [], []
    for rep in range(3):
        c_lat = torch.randn(B, h, h, 4, generator=g).cuda()
        hint = torch.randn(B, h, h, 256, generator=g).to(torch.bfloat16).cuda()
        noise = torch.randn(B, h, h, 4, generator=g).cuda()
        m.use_plans = False
        outs_eager.append(m.relay_decode_u8(c_lat, hint, ctx, noise, 2))
        m.use_plans = True
        outs_plan.append(m.relay_decode_u8(c_lat, hint, ctx, noise, 2))
    torch.cuda.synchronize()
    for a, b in zip(outs_eager, outs_plan):
        assert torch.equal(a, b)
    assert not torch.equal(outs_plan[0], outs_plan[1])  # inputs really changed between replays
    assert len(m._plans.plans) == 1
    plan = next(iter(m._plans.plans.values()))[0]
    assert len(plan) > 100
    ops.PROFILE, ops.PROFILE_OTHER = [], {}
    try:
        m.relay_decode_u8(c_lat, hint, ctx, noise, 2)
        torch.cuda.synchronize()
        n, flops, ms = ops.conv_profile_summary(ops.PROFILE)
        assert n > 100 and flops > 0 and ms > 0  # replay keeps per-kernel events for the roofline
        assert "attention" in ops.PROFILE_OTHER and "gn_stats" in ops.PROFILE_OTHER
    finally:
        ops.PROFILE, ops.PROFILE_OTHER = None, {}


def test_codec_plans_match_eager(gpu):
    """compress (VAE encoder + nets + stages + host rANS steps, two interleaved image groups) and
    decompress (stages with their rANS round trips) recorded as plans: byte-identical bitstreams and
    bit-identical latents vs the eager path, across replays with new images."""
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_image
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    m.preprocess_model.update(force=True)
    m.preprocess_model.coder_groups = 2
    B, S = 3, 128  # odd batch: unequal image groups
    for rep in range(3):
        imgs = torch.from_numpy(np.stack([synth_image(S, S, 500 + 10 * rep + i) for i in range(B)])).cuda()
        m.use_plans = False
        bodies_e = m.compress_images(imgs)
        lat_e, hint_e = m.decompress_bodies(bodies_e)
        m.use_plans = True
        bodies_p = m.compress_images(imgs)
        lat_p, hint_p = m.decompress_bodies(bodies_p)
        torch.cuda.synchronize()
        assert bodies_p == bodies_e
        assert torch.equal(lat_p, lat_e) and torch.equal(hint_p, hint_e)
    assert len(m.preprocess_model._plans.plans) == 2
    # one group (no interleave) gives the same bytes
    m.preprocess_model.coder_groups = 1
    assert m.compress_images(imgs) == bodies_e


def test_plan_pools_survive_cyclic_gc(gpu):
    """A plan and its tensors in a reference cycle, collected by a GC pass that runs inside another
    plan's recording (what aborted the round-1 driver run): the pool must outlive its tensors, and
    dead pools with no live block are released when the next plan is made."""
    import gc

    from rdeic_amd import plan

    class Owner:
        pass

    for _ in range(3):
        o, p = Owner(), plan.LaunchPlan()
        o.plan, p.owner = p, o  # cycle: only the cyclic GC frees it
        o.t = p.record(lambda: torch.ones(1 << 20, device="cuda"))
        del o, p
    live = plan.LaunchPlan()
    out = live.record(lambda: (gc.collect(), torch.full((1 << 20,), 2.0, device="cuda"))[1])
    torch.cuda.synchronize()
    assert float(out.sum()) == 2.0 * (1 << 20)
    plan.LaunchPlan()  # sweeps: the three collected plans' pools are free now
    dead = [pool for ref, pool in plan._POOLS if ref() is None]
    assert len(dead) <= 1, len(dead)  # at most the plan made just above
