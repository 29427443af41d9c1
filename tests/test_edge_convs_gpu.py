"""The VAE edge convolutions (rdeic_amd/csrc/conv_edge.hip; reference ldm/modules/diffusionmodules/model.py:556
Encoder.conv_in and :681-683 Decoder norm_out -> nonlinearity -> conv_out).

* conv_in (8 input channels, the image padded from 3): outputs and fused GroupNorm statistics bit-identical to the
  register tile it replaces (rdeic_set_conv_option(10, 0)), and within bf16 tolerance of torch fp32.
* norm -> SiLU -> conv to <= 16 channels: against torch fp32 on the bf16-rounded normalised input, and against the
  materialised path (GroupNorm apply kernel + tiny-cout conv) it replaces; batch invariance.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous().cuda()


def _nchw(x):
    return x.permute(0, 3, 1, 2).float().cpu()


def _conv_in_run(x8, p, stats, edge):
    from rdeic_amd import ops
    prev = ops.set_edge_conv(edge)
    try:
        c0 = ops.launch_count(ops.COUNT_EDGE)
        y = ops.conv2d(x8, p, stats=stats)
        ran = ops.launch_count(ops.COUNT_EDGE) > c0
        ab = None
        if stats:
            g = torch.Generator().manual_seed(5)
            gamma = (torch.rand(p.cout, generator=g) + 0.5).cuda()
            beta = torch.randn(p.cout, generator=g).cuda()
            ab = ops.group_norm_ab(y, gamma, beta, 32, 1e-6)
        torch.cuda.synchronize()
        return y, ab, ran
    finally:
        ops.set_edge_conv(prev)


@pytest.mark.parametrize("n,h,w,stats,cout", [(2, 64, 128, True, 128), (1, 40, 64, False, 128), (3, 16, 64, True, 64),
                                               (1, 512, 512, True, 128), (2, 8, 64, True, 96)])
def test_conv_in8_bit_identical_and_vs_torch(gpu, n, h, w, stats, cout):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(n * h + w)
    x = torch.rand(n, 3, h, w, generator=g) * 2 - 1
    wt = torch.randn(cout, 3, 3, 3, generator=g) / math.sqrt(27)
    b = torch.randn(cout, generator=g) * 0.1
    x8 = torch.zeros(n, h, w, 8)
    x8[..., :3] = x.permute(0, 2, 3, 1)
    x8 = x8.to(torch.bfloat16).cuda()
    w8 = torch.zeros(cout, 8, 3, 3)
    w8[:, :3] = wt
    p = ops.ConvParams.pack(w8, b, pad=1, dtype=torch.bfloat16)
    y1, ab1, ran1 = _conv_in_run(x8, p, stats, 1)
    y0, ab0, ran0 = _conv_in_run(x8, p, stats, 0)
    assert ran1 and not ran0
    assert torch.equal(y1, y0)
    if stats:
        assert torch.equal(ab1, ab0)
    ref = F.conv2d(x.to(torch.bfloat16).float(), wt.to(torch.bfloat16).float(), b, padding=1)
    torch.testing.assert_close(_nchw(y1), ref, rtol=1e-2, atol=1e-2)


def _narrow_ref(x, gamma, beta, wt, b, silu):
    xq = x.to(torch.bfloat16).float()
    hn = F.group_norm(xq, 32, gamma, beta, eps=1e-6)
    if silu:
        hn = F.silu(hn)
    return F.conv2d(hn.to(torch.bfloat16).float(), wt.to(torch.bfloat16).float(), b, padding=1)


@pytest.mark.parametrize("n,cin,cout,h,w,silu", [(2, 128, 3, 32, 64, True), (1, 256, 4, 16, 128, True),
                                                 (3, 64, 16, 40, 64, False), (1, 128, 3, 512, 512, True)])
def test_narrow_gn_conv_vs_torch_and_materialised(gpu, n, cin, cout, h, w, silu):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(cin * cout + h)
    x = torch.randn(n, cin, h, w, generator=g) * 2 + 1
    gamma, beta = torch.rand(cin, generator=g) + 0.5, torch.randn(cin, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g)
    xd = _nhwc(x.to(torch.bfloat16))
    ab = ops.group_norm_ab(xd, gamma.cuda(), beta.cuda(), 32, 1e-6)
    p = ops.ConvParams.pack(wt, b, pad=1, dtype=torch.bfloat16)
    outs = {}
    for edge in (1, 0):
        prev = ops.set_edge_conv(edge)
        try:
            c0 = ops.launch_count(ops.COUNT_EDGE)
            outs[edge] = ops.conv2d(xd, p, gn=ab, gn_silu=silu, out_f32=True)
            torch.cuda.synchronize()
            assert (ops.launch_count(ops.COUNT_EDGE) > c0) == bool(edge)
        finally:
            ops.set_edge_conv(prev)
    ref = _narrow_ref(x, gamma, beta, wt, b, silu)
    torch.testing.assert_close(_nchw(outs[1]), ref, rtol=1e-2, atol=2e-2)
    # the same GroupNorm + SiLU up to the rcp / IEEE-divide rounding of the bf16 inputs, summed in another order
    d = (outs[1] - outs[0]).abs().max().item()
    assert d <= 3e-3 * max(1.0, ref.abs().max().item()), d
    if n > 1:  # batch invariance: image 1 alone
        prev = ops.set_edge_conv(1)
        try:
            y1 = ops.conv2d(xd[1:2].contiguous(), p, gn=ab[1:2].contiguous(), gn_silu=silu, out_f32=True)
        finally:
            ops.set_edge_conv(prev)
        assert torch.equal(y1, outs[1][1:2])
