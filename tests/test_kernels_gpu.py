"""Kernel-level numerics on the MI355X: each HIP kernel against a plain PyTorch fp32 (CPU)
reference of the same op. fp32 parity mode must agree to ~1e-5 relative; bf16 mode to the
bf16 rounding of its inputs."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _nhwc(x):  # NCHW cpu -> NHWC cuda
    return x.permute(0, 2, 3, 1).contiguous().cuda()


def _nchw(x):
    return x.float().cpu().permute(0, 3, 1, 2)


def _tol(dtype):
    return (2e-5, 2e-5) if dtype == torch.float32 else (3e-2, 3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,stride,pad,h", [
    (64, 64, 3, 1, 1, 16), (128, 320, 3, 1, 1, 12), (320, 640, 3, 2, 1, 16), (4, 320, 3, 1, 1, 8),
    (256, 16, 5, 1, 2, 8), (48, 224, 5, 1, 2, 8), (512, 8, 1, 1, 0, 8), (260, 64, 3, 1, 1, 8),
    (3, 128, 3, 1, 1, 16), (256, 1024, 1, 1, 0, 4), (128, 3, 3, 1, 1, 16)])
def test_conv2d(gpu, dtype, cin, cout, k, stride, pad, h):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(cin * 1000 + cout)
    x = torch.randn(2, cin, h, h + 2, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)
    b = torch.randn(cout, generator=g)
    p = ops.ConvParams.pack(w, b, stride=stride, pad=pad, dtype=dtype)
    xq = x.to(dtype).float()
    wq = w.to(dtype).float()
    ref = F.conv2d(xq, wq, b, stride=stride, padding=pad)
    out = ops.conv2d(_nhwc(x.to(dtype)), p)
    torch.cuda.synchronize()
    rt, at = _tol(dtype)
    torch.testing.assert_close(_nchw(out), ref, rtol=rt, atol=at * ref.abs().max().item())


def test_conv2d_fp32_large_tile(gpu):
    """fp32 layers with >= 512 128x128 tiles (the VAE encoder at 512^2 in the fine-tune step) run
    the 128x128 tile: vs torch fp32, with GN/SiLU prologue and residual."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(11)
    x = torch.randn(1, 128, 256, 256, generator=g)
    w = torch.randn(128, 128, 3, 3, generator=g) / math.sqrt(128 * 9)
    b = torch.randn(128, generator=g)
    r = torch.randn(1, 128, 256, 256, generator=g)
    gamma, beta = torch.rand(128, generator=g) + 0.5, torch.randn(128, generator=g) * 0.1
    ref = F.conv2d(F.silu(F.group_norm(x, 32, gamma, beta, eps=1e-6)), w, b, padding=1) + r
    p = ops.ConvParams.pack(w, b, pad=1, dtype=torch.float32)
    xd = _nhwc(x)
    ab = ops.group_norm_ab(xd, gamma.cuda(), beta.cuda(), 32, 1e-6)
    out = ops.conv2d(xd, p, gn=ab, gn_silu=True, res=_nhwc(r))
    torch.testing.assert_close(_nchw(out), ref, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv2d_fusions(gpu, dtype):
    """concat + GN/SiLU prologue + emb + leaky + residual; up2; asymmetric pad; pixel shuffle."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(7)
    n, c1, c2, co, h = 2, 64, 32, 64, 8
    xa = torch.randn(n, c1, h, h, generator=g) * 2 + 1
    xb = torch.randn(n, c2, h, h, generator=g)
    w = torch.randn(co, c1 + c2, 3, 3, generator=g) / math.sqrt(9 * (c1 + c2))
    b = torch.randn(co, generator=g)
    emb = torch.randn(n, co, generator=g)
    res = torch.randn(n, co, h, h, generator=g)
    gamma = torch.rand(c1 + c2, generator=g) + 0.5
    beta = torch.randn(c1 + c2, generator=g) * 0.1
    xcat = torch.cat([xa, xb], 1)
    xq = xcat.to(dtype).float()
    gn = F.group_norm(xq, 32, gamma, beta, eps=1e-5)
    ref = F.conv2d(F.silu(gn).to(dtype).float(), w.to(dtype).float(), b, padding=1) + emb[:, :, None, None]
    ref = F.leaky_relu(ref, 0.1) + res.to(dtype).float()
    p = ops.ConvParams.pack(w, b, pad=1, dtype=dtype)
    xa_d, xb_d = _nhwc(xa.to(dtype)), _nhwc(xb.to(dtype))
    # GN stats over the concatenation: build it explicitly for the stats kernel
    xcat_d = _nhwc(xcat.to(dtype))
    ab = ops.group_norm_ab(xcat_d, gamma.cuda(), beta.cuda(), 32, 1e-5)
    out = ops.conv2d(xa_d, p, x2=xb_d, gn=ab, gn_silu=True, emb=emb.cuda(), act=ops.LEAKY, slope=0.1,
                     res=_nhwc(res.to(dtype)))
    torch.cuda.synchronize()
    rt, at = _tol(dtype)
    torch.testing.assert_close(_nchw(out), ref, rtol=rt, atol=at * 4)

    # nearest x2 upsample + conv
    wu = torch.randn(32, c1, 3, 3, generator=g) / math.sqrt(9 * c1)
    pu = ops.ConvParams.pack(wu, None, pad=1, dtype=dtype)
    refu = F.conv2d(F.interpolate(xa.to(dtype).float(), scale_factor=2, mode="nearest"), wu.to(dtype).float(),
                    padding=1)
    outu = ops.conv2d(xa_d, pu, up2=True)
    torch.testing.assert_close(_nchw(outu), refu, rtol=rt, atol=at * 4)

    # VAE downsample: pad (0,1,0,1) then stride-2 conv, pad 0
    pd = ops.ConvParams.pack(wu, None, stride=2, pad=0, dtype=dtype)
    refd = F.conv2d(F.pad(xa.to(dtype).float(), (0, 1, 0, 1)), wu.to(dtype).float(), stride=2)
    outd = ops.conv2d(xa_d, pd, pad_t=0, pad_l=0, out_hw=(h // 2, h // 2))
    torch.testing.assert_close(_nchw(outd), refd, rtol=rt, atol=at * 4)

    # subpel: 1x1 conv to 4C then PixelShuffle(2), leaky 0.01
    ws = torch.randn(4 * 16, c1, 1, 1, generator=g) / math.sqrt(c1)
    bs = torch.randn(4 * 16, generator=g)
    ps = ops.ConvParams.pack(ws, bs, dtype=dtype)
    refs = F.leaky_relu(F.pixel_shuffle(F.conv2d(xa.to(dtype).float(), ws.to(dtype).float(), bs), 2), 0.01)
    outs = ops.conv2d(xa_d, ps, pixel_shuffle=True, act=ops.LEAKY, slope=0.01)
    torch.testing.assert_close(_nchw(outs), refs, rtol=rt, atol=at * 4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c,groups,hw", [(128, 32, 64), (320, 32, 24), (1280, 32, 8), (64, 32, 40)])
def test_groupnorm(gpu, dtype, c, groups, hw):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(c + hw)
    x = torch.randn(2, c, hw, hw + 1, generator=g) * 3 + 5
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g)
    xq = x.to(dtype).float()
    ref = F.silu(F.group_norm(xq, groups, gamma, beta, eps=1e-6))
    xd = _nhwc(x.to(dtype))
    ab = ops.group_norm_ab(xd, gamma.cuda(), beta.cuda(), groups, 1e-6)
    out = ops.group_norm_apply(xd, ab, silu=True)
    torch.cuda.synchronize()
    rt, at = (1e-4, 1e-4) if dtype == torch.float32 else (2e-2, 2e-2)
    torch.testing.assert_close(_nchw(out), ref, rtol=rt, atol=at)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_layernorm_geglu(gpu, dtype):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(3)
    x = torch.randn(77, 320, generator=g) * 2 + 1
    gamma, beta = torch.rand(320, generator=g) + 0.5, torch.randn(320, generator=g)
    ref = F.layer_norm(x.to(dtype).float(), (320,), gamma, beta, 1e-5)
    out = ops.layer_norm(x.to(dtype).cuda(), gamma.cuda(), beta.cuda(), 1e-5)
    rt, at = (1e-5, 1e-5) if dtype == torch.float32 else (2e-2, 2e-2)
    torch.testing.assert_close(out.float().cpu(), ref, rtol=rt, atol=at)
    y = torch.randn(50, 2 * 96, generator=g)
    yq = y.to(dtype).float()
    refg = yq[:, :96] * F.gelu(yq[:, 96:])
    outg = ops.geglu(y.to(dtype).cuda())
    torch.testing.assert_close(outg.float().cpu(), refg, rtol=rt, atol=at)


def _ref_attn(q, k, v, heads, dh, scale):
    b, lq, _ = q.shape
    lk = k.shape[1]
    qh = q.view(b, lq, heads, dh).permute(0, 2, 1, 3)
    kh = k.view(b, lk, heads, dh).permute(0, 2, 1, 3)
    vh = v.view(b, lk, heads, dh).permute(0, 2, 1, 3)
    s = torch.einsum("bhid,bhjd->bhij", qh, kh) * scale
    o = torch.einsum("bhij,bhjd->bhid", s.softmax(-1), vh)
    return o.permute(0, 2, 1, 3).reshape(b, lq, heads * dh)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("heads,dh,lq,lk", [(5, 64, 256, 256), (4, 16, 300, 300), (10, 64, 64, 77), (16, 16, 64, 77),
                                           (4, 16, 4096, 4096), (8, 32, 130, 200), (2, 16, 1100, 77), (2, 32, 1030, 300),
                                           (20, 64, 100, 33), (2, 16, 2300, 2100), (3, 16, 2100, 77)])
def test_attention(gpu, dtype, heads, dh, lq, lk):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(heads * dh + lq)
    b = 2
    q = torch.randn(b, lq, heads * dh, generator=g)
    k = torch.randn(b, lk, heads * dh, generator=g)
    v = torch.randn(b, lk, heads * dh, generator=g)
    scale = dh ** -0.5
    ref = _ref_attn(q.to(dtype).float(), k.to(dtype).float(), v.to(dtype).float(), heads, dh, scale)
    qd = q.to(dtype).cuda().view(b * lq, -1)
    kd = k.to(dtype).cuda().view(b * lk, -1)
    vd = v.to(dtype).cuda().view(b * lk, -1)
    out = torch.empty_like(qd)
    ops.attention(qd, kd, vd, out, batch=b, heads=heads, lq=lq, lk=lk, dh=dh, scale=scale)
    torch.cuda.synchronize()
    rt, at = (2e-5, 2e-5) if dtype == torch.float32 else (3e-2, 3e-2)
    torch.testing.assert_close(out.float().cpu().view(b, lq, -1), ref, rtol=rt, atol=at)


@pytest.mark.parametrize("lq,lk", [(300, 1000), (2300, 2100)])
def test_attention_d16_running_max_moves(gpu, lq, lk):
    """d = 16 kernels (one and two query groups per wave): scores that grow along the keys, so the
    running max moves past its 2^8 slack many times (the ballot-gated rescale), plus a large
    dynamic range; bf16 against the fp32 reference."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(5)
    b, heads, dh = 2, 4, 16
    q = torch.randn(b, lq, heads * dh, generator=g) * 3
    ramp = torch.linspace(0.2, 6.0, lk).view(1, lk, 1)
    k = torch.randn(b, lk, heads * dh, generator=g) * ramp
    v = torch.randn(b, lk, heads * dh, generator=g)
    scale = dh ** -0.5
    qb, kb, vb = q.to(torch.bfloat16), k.to(torch.bfloat16), v.to(torch.bfloat16)
    ref = _ref_attn(qb.float(), kb.float(), vb.float(), heads, dh, scale)
    qd, kd, vd = (t.cuda().view(-1, heads * dh) for t in (qb, kb, vb))
    out = torch.empty_like(qd)
    ops.attention(qd, kd, vd, out, batch=b, heads=heads, lq=lq, lk=lk, dh=dh, scale=scale)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.float().cpu().view(b, lq, -1), ref, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_attention_materialized(gpu, dtype):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(11)
    b, L, d = 2, 256, 512
    q = torch.randn(b, L, d, generator=g)
    k = torch.randn(b, L, d, generator=g)
    v = torch.randn(b, L, d, generator=g)
    ref = _ref_attn(q.to(dtype).float(), k.to(dtype).float(), v.to(dtype).float(), 1, d, d ** -0.5)
    qd, kd, vd = (t.to(dtype).cuda().view(b * L, d) for t in (q, k, v))
    out = torch.empty_like(qd)
    ops.attention_single_head_materialized(qd, kd, vd, out, batch=b, length=L, dim=d, scale=d ** -0.5)
    torch.cuda.synchronize()
    rt, at = (1e-4, 1e-4) if dtype == torch.float32 else (3e-2, 3e-2)
    torch.testing.assert_close(out.float().cpu().view(b, L, d), ref, rtol=rt, atol=at)


def test_fill_uniform_matches_oracle(gpu):
    """The device weight generator is bit-identical to the CPU oracle generator."""
    from rdeic_amd import ops
    from oracle import weights_cpu
    n = 100003
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    ops.fill_uniform(out, 123456789, 0.05, 1.0)
    ref = weights_cpu.fill_uniform(n, 123456789, 0.05, 1.0)
    assert torch.equal(out.cpu(), torch.from_numpy(ref))


@pytest.mark.parametrize("c,hw", [(128, 45), (256, 33), (96, 70)])
def test_groupnorm_large_bf16(gpu, c, hw):
    """Several pass-1 chunks per image (unrolled pixel loop + tail), parallel finalize."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(c * hw)
    x = torch.randn(3, c, hw, hw + 3, generator=g) * 2 - 7
    gamma = torch.rand(c, generator=g) + 0.5
    beta = torch.randn(c, generator=g)
    xq = x.to(torch.bfloat16).float()
    ref = F.silu(F.group_norm(xq, 32, gamma, beta, eps=1e-6))
    xd = _nhwc(x.to(torch.bfloat16))
    ab = ops.group_norm_ab(xd, gamma.cuda(), beta.cuda(), 32, 1e-6)
    out = ops.group_norm_apply(xd, ab, silu=True)
    torch.testing.assert_close(_nchw(out), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("c", [320, 640, 1280, 1024])
def test_layernorm_vec(gpu, c):
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(c)
    x = torch.randn(301, c, generator=g) * 3 + 2
    gamma, beta = torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g)
    ref = F.layer_norm(x.to(torch.bfloat16).float(), (c,), gamma, beta, 1e-5)
    out = ops.layer_norm(x.to(torch.bfloat16).cuda(), gamma.cuda(), beta.cuda(), 1e-5)
    torch.testing.assert_close(out.float().cpu(), ref, rtol=2e-2, atol=3e-2)


@pytest.mark.parametrize("cout,h,w", [(3, 40, 37), (4, 16, 16), (1, 33, 20)])
def test_conv_small_cout_gn(gpu, cout, h, w):
    """Tiny-cout direct conv (VAE conv_out) with the GroupNorm + SiLU prologue."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(cout * h)
    cin = 128
    x = torch.randn(2, cin, h, w, generator=g) * 2 + 1
    gamma, beta = torch.rand(cin, generator=g) + 0.5, torch.randn(cin, generator=g)
    wt = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g)
    xq = x.to(torch.bfloat16).float()
    hn = F.silu(F.group_norm(xq, 32, gamma, beta, eps=1e-6)).to(torch.bfloat16).float()
    ref = F.conv2d(hn, wt.to(torch.bfloat16).float(), b, padding=1)
    xd = _nhwc(x.to(torch.bfloat16))
    ab = ops.group_norm_ab(xd, gamma.cuda(), beta.cuda(), 32, 1e-6)
    p = ops.ConvParams.pack(wt, b, pad=1, dtype=torch.bfloat16)
    out = ops.conv2d(xd, p, gn=ab, gn_silu=True, out_f32=True)
    torch.testing.assert_close(_nchw(out), ref, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("cin,cout,hw,res", [(1280, 1280, 8, True), (2560, 1280, 8, False), (640, 640, 16, True)])
def test_conv_splitk(gpu, cin, cout, hw, res):
    """Split-K conv (UNet 8x8 / 16x16 levels) vs the fp32 torch reference, with emb + act + residual."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(cin + hw)
    B = 16
    x = torch.randn(B, cin, hw, hw, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    b = torch.randn(cout, generator=g)
    emb = torch.randn(B, cout, generator=g)
    r = torch.randn(B, cout, hw, hw, generator=g)
    xq, wq, rq = x.to(torch.bfloat16).float(), w.to(torch.bfloat16).float(), r.to(torch.bfloat16).float()
    ref = F.silu(F.conv2d(xq, wq, b, padding=1) + emb[:, :, None, None])
    if res:
        ref = ref + rq
    p = ops.ConvParams.pack(w, b, pad=1, dtype=torch.bfloat16)
    xd, rd = _nhwc(x.to(torch.bfloat16)), _nhwc(r.to(torch.bfloat16))
    with ops.splitk_allowed():
        assert ops._splitk_count(xd, None, B * hw * hw, p, False, rd, B) > 1
        out = ops.conv2d(xd, p, emb=emb.cuda(), act=ops.SILU, res=rd if res else None)
    torch.testing.assert_close(_nchw(out), ref, rtol=2e-2, atol=3e-2)
    out_plain = ops.conv2d(xd, p, emb=emb.cuda(), act=ops.SILU, res=rd if res else None)
    assert (out.float() - out_plain.float()).abs().max().item() < 0.1


@pytest.mark.parametrize("cin,cout,hw,k,res", [(1280, 1280, 8, 3, True), (256, 256, 16, 3, False),
                                               (1280, 1280, 16, 1, True)])
def test_conv_splitk_fp32(gpu, cin, cout, hw, k, res):
    """fp32 split-K conv (the fine-tune step's B=1 small-M layers) vs torch fp32, and vs the
    unsplit fp32 kernel."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(cin + hw + k)
    x = torch.randn(1, cin, hw, hw, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)
    b = torch.randn(cout, generator=g)
    emb = torch.randn(1, cout, generator=g)
    r = torch.randn(1, cout, hw, hw, generator=g)
    ref = F.silu(F.conv2d(x, w, b, padding=k // 2) + emb[:, :, None, None])
    if res:
        ref = ref + r
    p = ops.ConvParams.pack(w, b, pad=k // 2, dtype=torch.float32)
    xd, rd = _nhwc(x), _nhwc(r)
    with ops.splitk_allowed(short_k=True):  # training: split counts from the real M (B=1)
        assert ops._splitk_count(xd, None, hw * hw, p, False, rd, 1) > 1
        out = ops.conv2d(xd, p, emb=emb.cuda(), act=ops.SILU, res=rd if res else None)
    assert out.dtype == torch.float32
    torch.testing.assert_close(_nchw(out), ref, rtol=1e-4, atol=1e-4)
    out_plain = ops.conv2d(xd, p, emb=emb.cuda(), act=ops.SILU, res=rd if res else None)
    torch.testing.assert_close(out, out_plain, rtol=1e-4, atol=5e-5)


@pytest.mark.parametrize("rows,cin,inner", [(4096, 320, 1280), (1000, 640, 2560), (256, 64, 256)])
def test_linear_fused_geglu(gpu, rows, cin, inner):
    """GEGLU in the projection's epilogue (conv out_mode 2, weights interleaved by
    ParamStore.conv_geglu) vs the unfused projection + rdeic_geglu and vs torch fp32."""
    from rdeic_amd import ops
    from rdeic_amd.params import ParamStore
    g = torch.Generator().manual_seed(rows + cin)
    x = torch.randn(rows, cin, generator=g)
    w = torch.randn(2 * inner, cin, generator=g) / math.sqrt(cin)
    b = torch.randn(2 * inner, generator=g) * 0.1
    st = ParamStore(torch.bfloat16, "cuda")
    st.shapes["ff.weight"], st.shapes["ff.bias"] = tuple(w.shape), tuple(b.shape)
    st.t["ff.weight"], st.t["ff.bias"] = w.cuda(), b.cuda()
    xb = x.to(torch.bfloat16).cuda()
    fused = ops.linear(xb, st.conv_geglu("ff"), geglu=True, images=1)
    unfused = ops.geglu(ops.linear(xb, st.conv("ff"), images=1))
    assert fused.shape == (rows, inner)
    assert (fused.float() - unfused.float()).abs().max().item() <= 2e-2 * unfused.float().abs().max().item()
    h = x.to(torch.bfloat16).float() @ w.to(torch.bfloat16).float().t() + b
    ref = h[:, :inner] * F.gelu(h[:, inner:])
    err = (fused.float().cpu() - ref).abs().max().item()
    assert err <= 3e-2 * ref.abs().max().item(), err
    with pytest.raises(ValueError):
        ops.linear(xb, st.conv_geglu("ff"), geglu=True, act=ops.GELU, images=1)



@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("heads,lq,lk,bcast", [(5, 4096, 4096, False), (10, 300, 77, True), (2, 130, 1000, False)])
def test_attention_dh64_kernels(gpu, mode, heads, lq, lk, bcast):
    """The register-staged (1) and LDS-DMA (2) head-dim-64 kernels vs torch fp32 (ragged tiles,
    broadcast K/V, long keys)."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(lq + lk)
    B, dh = 2, 64
    q = torch.randn(B, lq, heads * dh, generator=g)
    kb = 1 if bcast else B
    k = torch.randn(kb, lk, heads * dh, generator=g)
    v = torch.randn(kb, lk, heads * dh, generator=g)
    qc, kc, vc = (t.to(torch.bfloat16).cuda() for t in (q, k, v))
    o = torch.empty(B * lq, heads * dh, dtype=torch.bfloat16, device="cuda")
    prev = ops.set_conv_option(1, mode)
    try:
        ops.attention(qc.view(-1, heads * dh), kc.view(-1, heads * dh), vc.view(-1, heads * dh), o, batch=B,
                      heads=heads, lq=lq, lk=lk, dh=dh, scale=dh ** -0.5, kv_bcast=bcast)
    finally:
        ops.set_conv_option(1, prev)
    qf, kf, vf = (t.to(torch.bfloat16).float() for t in (q, k, v))
    ref = _ref_attn(qf, kf.expand(B, -1, -1).contiguous(), vf.expand(B, -1, -1).contiguous(), heads, dh, dh ** -0.5)
    err = (o.float().cpu().view(B, lq, -1) - ref).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("rows,cin,couts,geglu", [(4096, 320, (320, 320, 320), False), (1024, 640, (640,), False),
                                                  (512, 1280, (2 * 5120,), True), (77 * 3, 320, (320,), False)])
def test_layernorm_folded_linear(gpu, rows, cin, couts, geglu):
    """LayerNorm folded into the linear it feeds (ParamStore.conv_ln + rdeic_layernorm_rowstats, the bf16
    transformer's norm1/2/3 -> to_qkv / to_q / ff.net.0.proj, attention.py:273-285): against the
    materialised LayerNorm + linear and against torch fp32 LayerNorm + Linear."""
    import torch.nn.functional as F
    from rdeic_amd import ops
    from rdeic_amd.params import ParamStore
    g = torch.Generator().manual_seed(rows + cin)
    x = (torch.randn(rows, cin, generator=g) * 1.7 + 0.4).to(torch.bfloat16)
    gamma = 1 + 0.3 * torch.randn(cin, generator=g)
    beta = 0.2 * torch.randn(cin, generator=g)
    st = ParamStore(torch.bfloat16, "cuda")
    names = []
    ws, bs = [], []
    for i, co in enumerate(couts):
        w = torch.randn(co, cin, generator=g) / math.sqrt(cin)
        b = torch.randn(co, generator=g) * 0.1
        st.shapes[f"l{i}.weight"], st.shapes[f"l{i}.bias"] = tuple(w.shape), tuple(b.shape)
        st.t[f"l{i}.weight"], st.t[f"l{i}.bias"] = w.cuda(), b.cuda()
        names.append(f"l{i}")
        ws.append(w)
        bs.append(b)
    st.shapes["ln.weight"] = st.shapes["ln.bias"] = (cin,)
    st.t["ln.weight"], st.t["ln.bias"] = gamma.cuda(), beta.cuda()
    xd = x.cuda()
    ops.launch_count_reset()
    ms = ops.layer_norm_rowstats(xd)
    fused = ops.linear(xd, st.conv_ln(names, "ln", geglu=geglu), ln_rows=ms, geglu=geglu, images=1)
    assert ops.launch_count(ops.COUNT_LN_FUSED) == 1 and ops.launch_count(ops.COUNT_LAYERNORM) == 0
    n = ops.layer_norm(xd, gamma.cuda(), beta.cuda())
    if geglu:
        unf = ops.linear(n, st.conv_geglu(names[0]), geglu=True, images=1)
    else:
        unf = ops.linear(n, st.conv_cat(names), images=1)
    torch.cuda.synchronize()
    # statistics: torch's LayerNorm of the bf16 rows in fp32
    xf = x.float()
    mean, var = xf.mean(1), xf.var(1, unbiased=False)
    torch.testing.assert_close(ms.cpu()[:, 0], mean, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(ms.cpu()[:, 1], torch.rsqrt(var + 1e-5), rtol=1e-5, atol=1e-5)
    nf = F.layer_norm(xf, (cin,), gamma, beta, 1e-5)
    h = nf @ torch.cat(ws).t() + torch.cat(bs)
    ref = h[:, : h.shape[1] // 2] * F.gelu(h[:, h.shape[1] // 2:]) if geglu else h
    scale = ref.abs().max().item()
    e_f = (fused.float().cpu() - ref).abs()
    e_u = (unf.float().cpu() - ref).abs()
    print(f"folded: max {e_f.max().item():.3e} mean {e_f.mean().item():.3e}; materialised: max {e_u.max().item():.3e} "
          f"mean {e_u.mean().item():.3e} (ref max {scale:.2f})")
    assert e_f.max().item() <= 2e-2 * scale
    assert e_f.mean().item() <= 1.5 * e_u.mean().item() + 1e-4  # no worse than the bf16 materialised path


@pytest.mark.parametrize("cin,cout,hw,B,act,res,emb,f32", [(1280, 1280, 8, 16, 3, True, True, False),
                                                         (2560, 1280, 8, 16, 0, False, False, False),
                                                         (640, 640, 16, 4, 3, True, True, False),
                                                         (1280, 640, 8, 3, 0, True, False, True)])
def test_conv_splitk_repeatable_with_stats(gpu, cin, cout, hw, B, act, res, emb, f32):
    """The split-K conv (LDS-DMA partial launch + the fixed-order reduce kernel) with its epilogue (emb, act,
    residual, fp32 output) and the output's GroupNorm statistics: two launches are bit-identical, and the
    statistics give the same affine as a standalone pass over the output."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(cin + cout + hw + B)
    x = _nhwc(torch.randn(B, cin, hw, hw, generator=g).to(torch.bfloat16))
    w = torch.randn(cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)
    p = ops.ConvParams.pack(w, torch.randn(cout, generator=g), pad=1, dtype=torch.bfloat16)
    e = torch.randn(B, cout, generator=g).cuda() if emb else None
    rd = _nhwc(torch.randn(B, cout, hw, hw, generator=g).to(torch.float32 if f32 else torch.bfloat16)) if res else None
    gamma, beta = torch.ones(cout, device="cuda"), torch.zeros(cout, device="cuda")
    outs = []
    for _ in range(2):
        with ops.splitk_allowed():
            assert ops._splitk_count(x, None, B * hw * hw, p, False, rd if rd is not None else x, B) > 1
            c0 = ops.launch_count(ops.COUNT_SPLITK)
            y = ops.conv2d(x, p, emb=e, act=act, res=rd, out_f32=f32, stats=not f32)
            assert ops.launch_count(ops.COUNT_SPLITK) == c0 + 1
        ab = None if f32 else ops.group_norm_ab(y, gamma, beta, 32, 1e-5)
        outs.append((y.clone(), ab))
    torch.cuda.synchronize()
    for y, ab in outs[1:]:
        assert torch.equal(outs[0][0], y)
        if ab is not None:
            assert torch.equal(outs[0][1], ab)


@pytest.mark.parametrize("levels,sorted_table", [(64, True), (64, False), (300, True), (2, True)])
def test_ckbd_indexes_scale_table(gpu, levels, sorted_table):
    """rdeic_ckbd_indexes / rdeic_ckbd_encode build_indexes (compressai GaussianConditional: L-1 - #{k: max(s, b) <=
    table[k]}): the LDS table's binary search on a non-decreasing table and the linear count on any other table
    (and on tables past the LDS capacity) give the reference's integers exactly, ties at table values included."""
    from rdeic_amd import ops
    g = torch.Generator().manual_seed(levels * 3 + int(sorted_table))
    n, hy, wy, c = 2, 6, 8, 5
    tab = torch.exp(torch.linspace(math.log(0.11), math.log(256.0), levels - 1))
    if not sorted_table:
        tab = tab[torch.randperm(levels - 1, generator=g)]
    # scales: random, exact table values (ties) and values below the bound
    scale = torch.exp(torch.rand(n, hy, wy, c, generator=g) * 7 - 3)
    flat = scale.view(-1)
    flat[::7] = tab[torch.randint(0, levels - 1, (flat[::7].numel(),), generator=g)]
    flat[::11] = 0.01
    params = torch.cat([scale, torch.randn(n, hy, wy, c, generator=g)], dim=3).contiguous()
    y = torch.randn(n, hy, wy, c, generator=g) * 3
    bound = 0.11
    wq = wy // 2
    for phase in (0, 1):
        idx = torch.full((n, c * hy * wq), -1, dtype=torch.int32, device="cuda")
        sym = torch.zeros_like(idx)
        yhat = torch.zeros(n, hy, wy, c, device="cuda")
        tab_d = tab.float().cuda()
        ops.call("rdeic_ckbd_indexes", params.cuda().data_ptr(), 2 * c, n, hy, wy, c, phase, tab_d.data_ptr(), levels,
                 bound, idx.data_ptr(), c * hy * wq, 0, 0, ops.stream_ptr())
        idx2 = torch.full_like(idx, -1)
        yc, pc = y.cuda(), params.cuda()
        ops.call("rdeic_ckbd_encode", yc.data_ptr(), c, pc.data_ptr(), 2 * c, n, hy, wy, c, phase, tab_d.data_ptr(),
                 levels, bound, sym.data_ptr(), idx2.data_ptr(), c * hy * wq, 0, yhat.data_ptr(), c, None, 0, 0,
                 ops.stream_ptr())
        torch.cuda.synchronize()
        # reference over the squeezed lattice [c][hy][wy/2]
        r = torch.arange(hy).view(hy, 1)
        j = torch.arange(wq).view(1, wq)
        col = (2 * j + 1 - (r & 1)) if phase == 0 else (2 * j + (r & 1))
        s = scale[:, r, col, :].permute(0, 3, 1, 2).reshape(n, -1)  # [n][c][hy][wq]
        s = torch.clamp(s, min=bound)
        ref = (levels - 1) - (s.unsqueeze(-1) <= tab.view(1, 1, -1)).sum(-1)
        assert torch.equal(idx.cpu().long(), ref.long())
        assert torch.equal(idx2.cpu().long(), ref.long())
