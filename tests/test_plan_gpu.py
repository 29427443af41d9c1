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
