"""GroupNorm statistics fused into the producing conv's epilogue (rdeic_conv_desc.gn_part ->
rdeic_groupnorm_parts_ab) against the stand-alone statistics pass over the same tensor
(rdeic_groupnorm_stats), for the GroupNorm sites of the path: ResnetBlock / ResBlock convs
(openaimodel.py:254-274; model.py:131-151), a skip concat (openaimodel.py:790-794), a
SpatialTransformer / AttnBlock proj_out linear (attention.py:345-350; model.py:181-205) and the
split-K fallback. The fused statistics are tile- and batch-invariant (canonical order), so the
affine of one image is bit-identical whatever else is in the batch."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def _conv(cin, cout, k=3, seed=0):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(seed)
    w = (torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)).cuda()
    b = (torch.randn(cout, generator=g) * 0.1).cuda()
    return ops.ConvParams.pack(w, b, pad=k // 2)


def _gamma_beta(c, seed=1):
    g = torch.Generator().manual_seed(seed)
    return (1 + 0.1 * torch.randn(c, generator=g)).cuda(), (0.1 * torch.randn(c, generator=g)).cuda()


def _standalone(x, gamma, beta, groups, eps, x2=None):
    from rdeic_amd import ops
    xc = x.clone()  # a fresh tensor object: no fused statistics attached
    x2c = None if x2 is None else x2.clone()
    return ops.group_norm_ab(xc, gamma, beta, groups, eps, x2=x2c)


@pytest.mark.parametrize("shape", [(2, 64, 64, 128, 128), (2, 32, 32, 320, 640), (3, 16, 16, 640, 1280),
                                   (2, 128, 128, 256, 256)])
def test_fused_stats_match_standalone(gpu, shape):
    from rdeic_amd import ops
    n, h, w, cin, cout = shape
    x = (torch.randn(n, h, w, cin, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    p = _conv(cin, cout)
    res = (torch.randn(n, h, w, cout, device="cuda") * 3 + 1).to(torch.bfloat16)
    y = ops.conv2d(x, p, res=res, stats=True)
    assert getattr(y, "_rdeic_gn_part", None) is not None
    gamma, beta = _gamma_beta(cout)
    ab_f = ops.group_norm_ab(y, gamma, beta, 32, 1e-5)
    ab_s = _standalone(y, gamma, beta, 32, 1e-5)
    torch.testing.assert_close(ab_f, ab_s, rtol=2e-4, atol=2e-5)


def test_fused_stats_batch_and_tile_invariant(gpu):
    from rdeic_amd import ops
    x = torch.randn(4, 64, 64, 256, device="cuda").to(torch.bfloat16)
    p = _conv(256, 256)
    gamma, beta = _gamma_beta(256)
    ab_b = ops.group_norm_ab(ops.conv2d(x, p, stats=True), gamma, beta, 32, 1e-6)
    ab_1 = ops.group_norm_ab(ops.conv2d(x[2:3].contiguous(), p, stats=True), gamma, beta, 32, 1e-6)
    assert torch.equal(ab_b[2:3], ab_1)
    for t in (3, 20, 24, 25, 26, 32, 34):  # register tile (fallback pass), LDS-DMA tiles (fused or not)
        ops.FORCE_TILE = t
        try:
            ab_t = ops.group_norm_ab(ops.conv2d(x, p, stats=True), gamma, beta, 32, 1e-6)
        finally:
            ops.FORCE_TILE = None
        assert torch.equal(ab_t, ab_b), t


def test_fused_stats_concat_linear_and_splitk(gpu):
    from rdeic_amd import ops
    # skip concat: GroupNorm over cat(h, skip) with both halves carrying statistics (30 ch/group
    # straddles the boundary at 640)
    h = ops.conv2d(torch.randn(2, 32, 32, 320, device="cuda").to(torch.bfloat16), _conv(320, 640, seed=2), stats=True)
    sk = ops.conv2d(torch.randn(2, 32, 32, 320, device="cuda").to(torch.bfloat16), _conv(320, 320, seed=3),
                    stats=True)
    gamma, beta = _gamma_beta(960)
    ab_f = ops.group_norm_ab(h, gamma, beta, 32, 1e-5, x2=sk)
    torch.testing.assert_close(ab_f, _standalone(h, gamma, beta, 32, 1e-5, x2=sk), rtol=2e-4, atol=2e-5)
    # a transformer's proj_out: token rows [B*L, C] -> NHWC view with the statistics
    B, H, W, C = 2, 32, 32, 640
    t_in = torch.randn(B * H * W, C, device="cuda").to(torch.bfloat16)
    r = torch.randn(B * H * W, C, device="cuda").to(torch.bfloat16)
    out = ops.tokens_to_nhwc(ops.linear(t_in, _conv(C, C, k=1, seed=4), res=r, stats_hw=H * W, images=B), B, H, W)
    gamma, beta = _gamma_beta(C)
    ab_f = ops.group_norm_ab(out, gamma, beta, 32, 1e-6)
    torch.testing.assert_close(ab_f, _standalone(out, gamma, beta, 32, 1e-6), rtol=2e-4, atol=2e-5)
    # split-K (UNet 8x8 level): the statistics come from the stand-alone partial pass
    x = torch.randn(16, 8, 8, 1280, device="cuda").to(torch.bfloat16)
    with ops.splitk_allowed():
        y = ops.conv2d(x, _conv(1280, 1280, seed=5), stats=True)
    gamma, beta = _gamma_beta(1280)
    ab_f = ops.group_norm_ab(y, gamma, beta, 32, 1e-5)
    torch.testing.assert_close(ab_f, _standalone(y, gamma, beta, 32, 1e-5), rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("n,h,c0,c1,groups,silu", [(3, 16, 1280, 0, 32, True), (2, 8, 1280, 640, 32, True),
                                                   (2, 16, 640, 640, 32, False), (4, 8, 320, 0, 16, True),
                                                   (1, 16, 2560, 0, 32, True), (2, 8, 640, 1280, 32, True)])
def test_parts_apply_bit_identical(gpu, n, h, c0, c1, groups, silu):
    """rdeic_groupnorm_parts_apply (the UNet's 16^2 / 8^2 GroupNorms: finalize + apply in one launch, through
    group_norm_ab(defer=True) -> conv2d(gn=...)) against the two-launch form (parts_ab, then the apply kernel):
    the affine and the normalised conv input are bit-identical, including a skip concat whose groups straddle the
    segments."""
    from rdeic_amd import ops
    xa = (torch.randn(n, h, h, 256, device="cuda") * 2 + 0.5).to(torch.bfloat16)
    ya = ops.conv2d(xa, _conv(256, c0, seed=3), stats=True)
    yb = ops.conv2d(xa, _conv(256, c1, seed=4), stats=True) if c1 else None
    gamma, beta = _gamma_beta(c0 + c1, seed=7)
    pc = _conv(c0 + c1, 128, k=1, seed=5)
    c_before = ops.launch_count(ops.COUNT_GN_PARTS_APPLY)
    ab_d = ops.group_norm_ab(ya, gamma, beta, groups, 1e-5, x2=yb, defer=True)
    assert getattr(ab_d, "_rdeic_pending", None) is not None
    out_d = ops.conv2d(ya, pc, x2=yb, gn=ab_d, gn_silu=silu)
    torch.cuda.synchronize()
    assert ops.launch_count(ops.COUNT_GN_PARTS_APPLY) == c_before + 1
    assert getattr(ab_d, "_rdeic_pending", None) is None
    ab_n = ops.group_norm_ab(ya, gamma, beta, groups, 1e-5, x2=yb)
    out_n = ops.conv2d(ya, pc, x2=yb, gn=ab_n, gn_silu=silu)
    torch.cuda.synchronize()
    assert torch.equal(ab_d, ab_n)
    assert torch.equal(out_d, out_n)


def test_parts_apply_deferred_affine_finalized_for_other_consumers(gpu):
    """A deferred affine read by anything but the materialised GroupNorm (here the apply kernel directly) is
    finalized first."""
    from rdeic_amd import ops
    xa = torch.randn(2, 16, 16, 256, device="cuda").to(torch.bfloat16)
    y = ops.conv2d(xa, _conv(256, 320, seed=9), stats=True)
    gamma, beta = _gamma_beta(320, seed=2)
    ab_d = ops.group_norm_ab(y, gamma, beta, 32, 1e-5, defer=True)
    o_d = ops.group_norm_apply(y, ab_d, silu=True)
    ab_n = ops.group_norm_ab(y, gamma, beta, 32, 1e-5)
    o_n = ops.group_norm_apply(y, ab_n, silu=True)
    assert torch.equal(ab_d, ab_n) and torch.equal(o_d, o_n)
