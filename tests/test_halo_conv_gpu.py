"""The 3x3 halo-strip conv with the input GroupNorm + SiLU applied in LDS (conv3x3_halo_kernel) — the
VAE ResnetBlock's norm -> nonlinearity -> conv (ldm/modules/diffusionmodules/model.py:131-151) —
against (a) the materialised path (rdeic_groupnorm_apply, then the im2col conv) within bf16
accumulation-order tolerance, (b) a torch fp32 reference of conv(silu(gn(x))), and for the
properties the path relies on: batch invariance (bit for bit), fused GroupNorm statistics of the
output equal to the stand-alone pass over it, residual / bias epilogue, the image-border zero
padding of the NORMALISED tensor, and the plain (no GroupNorm) variant."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _params(cin, cout, seed):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g) * 0.1
    return w, b, ops.ConvParams.pack(w.cuda(), b.cuda(), pad=1)


def _gn_ab(x, groups, seed, eps=1e-6):
    from rdeic_amd import ops
    c = x.shape[3]
    g = torch.Generator().manual_seed(seed)
    gamma = (1 + 0.2 * torch.randn(c, generator=g)).cuda()
    beta = (0.2 * torch.randn(c, generator=g)).cuda()
    return ops.group_norm_ab(x.clone(), gamma, beta, groups, eps)


def _run(x, p, ab, silu=True, res=None, stats=False, halo=True):
    from rdeic_amd import ops
    prev = ops.set_halo_conv(1 if halo else 0)
    prev_c, ops.HALO_MAX_C = ops.HALO_MAX_C, 512  # every width the kernel supports, not only the ones it wins
    try:
        n0 = ops.launch_count(ops.COUNT_HALO_CONV)
        y = ops.conv2d(x, p, gn=ab, gn_silu=silu, res=res, stats=stats)
        # the library's own dispatch took the halo kernel (not a silent fallback to the apply + im2col path)
        assert (ops.launch_count(ops.COUNT_HALO_CONV) > n0) == halo
        return y
    finally:
        ops.set_halo_conv(prev)
        ops.HALO_MAX_C = prev_c


@pytest.mark.parametrize("n,h,w,cin,cout", [(2, 64, 128, 128, 128), (1, 32, 64, 256, 128), (2, 16, 64, 128, 256),
                                            (1, 8, 64, 512, 512), (3, 4, 192, 64, 128)])
def test_halo_gn_conv_vs_materialised_and_torch(gpu, n, h, w, cin, cout):
    torch.manual_seed(n * h + cin)
    x = (torch.randn(n, h, w, cin, device="cuda") * 1.5 + 0.3).to(torch.bfloat16)
    wt, b, p = _params(cin, cout, seed=cin + cout)
    ab = _gn_ab(x, 32, seed=7)
    res = torch.randn(n, h, w, cout, device="cuda").to(torch.bfloat16)
    y_h = _run(x, p, ab, res=res)
    y_m = _run(x, p, ab, res=res, halo=False)
    torch.cuda.synchronize()
    # same bf16 inputs to the MFMAs (the in-LDS transform reproduces rdeic_groupnorm_apply's values);
    # only the fp32 accumulation order differs
    d = (y_h.float() - y_m.float()).abs()
    assert d.max().item() <= 2e-2 * max(1.0, y_m.float().abs().max().item()), d.max().item()
    # torch fp32: conv(silu(x * a + b)) + bias + res, on the bf16-rounded normalised input
    a_, b_ = ab[..., 0].cpu(), ab[..., 1].cpu()
    xn = x.float().cpu() * a_[:, None, None, :] + b_[:, None, None, :]
    xn = (xn * torch.sigmoid(xn)).to(torch.bfloat16).float()
    ref = F.conv2d(xn.permute(0, 3, 1, 2), wt.to(torch.bfloat16).float(), b, padding=1).permute(0, 2, 3, 1)
    ref = ref + res.float().cpu()
    err = (y_h.float().cpu() - ref).abs()
    assert err.max().item() < 3e-2 * max(1.0, ref.abs().max().item()), err.max().item()
    assert err.mean().item() < 3e-3, err.mean().item()


def test_halo_conv_batch_invariant_and_plain(gpu):
    from rdeic_amd import ops
    x = torch.randn(3, 32, 64, 128, device="cuda").to(torch.bfloat16)
    _, _, p = _params(128, 128, seed=3)
    ab = _gn_ab(x, 32, seed=5)
    y = _run(x, p, ab)
    y1 = _run(x[1:2].contiguous(), p, ab[1:2].contiguous())
    assert torch.equal(y[1:2], y1)
    # no GroupNorm (mode 2 routes every eligible conv to the halo kernel): vs the im2col conv
    prev = ops.set_halo_conv(2)
    try:
        yp = ops.conv2d(x, p)
    finally:
        ops.set_halo_conv(prev)
    ym = ops.conv2d(x, p)
    assert (yp.float() - ym.float()).abs().max().item() < 2e-2 * max(1.0, ym.float().abs().max().item())


def test_halo_conv_fused_output_statistics(gpu):
    """The output's GroupNorm statistics come out of the halo kernel's epilogue (64-pixel wave rows
    = canonical 64-row blocks): equal to the stand-alone statistics pass over the same tensor."""
    from rdeic_amd import ops
    x = torch.randn(2, 64, 128, 128, device="cuda").to(torch.bfloat16)
    _, _, p = _params(128, 256, seed=11)
    ab = _gn_ab(x, 32, seed=2)
    y = _run(x, p, ab, stats=True)
    assert getattr(y, "_rdeic_gn_part", None) is not None
    g = torch.Generator().manual_seed(4)
    gamma, beta = (1 + 0.1 * torch.randn(256, generator=g)).cuda(), (0.1 * torch.randn(256, generator=g)).cuda()
    ab_f = ops.group_norm_ab(y, gamma, beta, 32, 1e-6)
    ab_s = ops.group_norm_ab(y.clone(), gamma, beta, 32, 1e-6)
    torch.testing.assert_close(ab_f, ab_s, rtol=2e-4, atol=2e-5)


def test_halo_conv_zero_padding_is_of_the_normalised_tensor(gpu):
    """silu(a * 0 + b) != 0: the conv's padding must be zeros of the NORMALISED input, so border
    outputs must match the materialised path even with a large GroupNorm shift."""
    x = torch.randn(1, 8, 64, 64, device="cuda").to(torch.bfloat16)
    _, _, p = _params(64, 128, seed=9)
    ab = _gn_ab(x, 32, seed=1)
    ab[..., 1] += 3.0  # large shift: silu(b) far from 0 outside the image if padding were wrong
    y_h = _run(x, p, ab)
    y_m = _run(x, p, ab, halo=False)
    d = (y_h.float() - y_m.float()).abs()
    assert d[:, 0].max().item() < 2e-2 * max(1.0, y_m.float().abs().max().item())
    assert d[:, :, 0].max().item() < 2e-2 * max(1.0, y_m.float().abs().max().item())


@pytest.mark.parametrize("n,h,w,cin,cout,silu", [(2, 16, 128, 128, 128, True), (1, 8, 64, 512, 512, True),
                                                 (2, 24, 64, 96, 256, False)])
def test_halo8_bit_identical_to_halo4(gpu, n, h, w, cin, cout, silu):
    """The 8-row halo conv (one 1024-thread block per CU, rdeic_set_conv_option(9, 1)) uses the 4-row
    kernel's MFMA order: outputs, residual epilogue and fused statistics are bit-identical."""
    from rdeic_amd import ops
    torch.manual_seed(h * cin + cout)
    x = (torch.randn(n, h, w, cin, device="cuda") * 1.3 - 0.2).to(torch.bfloat16)
    _, _, p = _params(cin, cout, seed=cin * 7 + cout)
    ab = _gn_ab(x, 32, seed=11)
    res = torch.randn(n, h, w, cout, device="cuda").to(torch.bfloat16)
    outs = []
    for mode in (1, 0):
        prev = ops.set_conv_option(9, mode)
        try:
            y = _run(x, p, ab, silu=silu, res=res, stats=True)
            gamma, beta = torch.ones(cout, device="cuda"), torch.zeros(cout, device="cuda")
            outs.append((y, ops.group_norm_ab(y, gamma, beta, 32, 1e-6)))
        finally:
            ops.set_conv_option(9, prev)
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
