"""Backward kernels of the fine-tune step (train.hip via rdeic_amd/autograd.py) against plain
PyTorch fp32 autograd references of the same ops, on the GPU, in fp32 parity mode (and bf16 where
the training path runs bf16). Tolerances are written per test."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _nhwc(t):
    return t.permute(0, 2, 3, 1).contiguous()


def _nchw(t):
    return t.permute(0, 3, 1, 2)


def _rel(a, b):
    a, b = a.detach().float(), b.detach().float()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("layout", ["nn", "tn", "nt", "tt"])
@pytest.mark.parametrize("shape", [(70, 130, 100, 3, 4), (260, 390, 200, 20, 32)],
                         ids=["tile64", "tile128"])  # (m, n, k, batch, split-K planes); ragged edges
def test_gemm_strided(gpu, dt, layout, shape):
    from rdeic_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(1)
    m, n, k, nb, planes = shape
    A = torch.randn((nb, m, k), device="cuda", generator=g)
    B = torch.randn((nb, k, n), device="cuda", generator=g)
    ref = torch.bmm(A.to(dt).float(), B.to(dt).float())
    a_st = A if layout[0] == "n" else A.transpose(1, 2).contiguous()   # "t": stored k-major
    b_st = B if layout[1] == "n" else B.transpose(1, 2).contiguous()
    a_st, b_st = a_st.to(dt), b_st.to(dt)
    a_sm, a_sk = (k, 1) if layout[0] == "n" else (1, m)
    b_sk, b_sn = (n, 1) if layout[1] == "n" else (1, k)
    C = torch.empty((nb, m, n), device="cuda", dtype=torch.float32)
    AG.gemm(a_st, 0, a_sm, a_sk, b_st, 0, b_sk, b_sn, C, 0, n, m=m, n=n, k=k, batch=nb, a_bs=(m * k, 0),
            b_bs=(k * n, 0), c_bs=(m * n, 0))
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert _rel(C, ref) < tol
    # split-K planes sum to the product
    ks = -(-k // planes)
    P = torch.empty((planes, m, n), device="cuda", dtype=torch.float32)
    R = torch.empty((planes, m), device="cuda", dtype=torch.float32)  # row sums of A (bias gradients)
    AG.gemm(a_st[0], 0, a_sm, a_sk, b_st[0], 0, b_sk, b_sn, P, 0, n, m=m, n=n, k=k, batch=planes, c_bs=(m * n, 0),
            ksplit=ks, rsum=R, rsum_bs=m)
    assert _rel(P.sum(0), ref[0]) < tol
    assert _rel(R.sum(0), A[0].to(dt).float().sum(1)) < tol


CONV_CASES = [
    # cin, cout, k, stride, pad, up2, pixel_shuffle, act, slope, emb, res
    (16, 24, 3, 1, 1, False, False, 0, 0.0, True, True),
    (24, 16, 3, 2, 1, False, False, 1, 0.01, False, False),
    (16, 32, 1, 2, 0, False, False, 0, 0.0, False, False),
    (8, 16, 5, 1, 2, False, False, 2, 0.0, False, False),
    (32, 32, 3, 1, 1, True, False, 0, 0.0, False, False),
    (16, 64, 1, 1, 0, False, True, 1, 0.01, False, True),
    (64, 40, 3, 1, 1, False, False, 1, 0.1, False, True),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_backward(gpu, case):
    from rdeic_amd import autograd as AG
    cin, cout, k, stride, pad, up2, ps, act, slope, use_emb, use_res = case
    g = torch.Generator(device="cuda").manual_seed(2)
    n, h, w = 2, 12, 10
    x = torch.randn((n, cin, h, w), device="cuda", generator=g)
    W = torch.randn((cout, cin, k, k), device="cuda", generator=g) / math.sqrt(cin * k * k)
    b = torch.randn(cout, device="cuda", generator=g) * 0.1
    emb = torch.randn((n, cout), device="cuda", generator=g) if use_emb else None
    xr, Wr, br = (t.clone().requires_grad_(True) for t in (x, W, b))
    er = emb.clone().requires_grad_(True) if use_emb else None
    xi = F.interpolate(xr, scale_factor=2.0, mode="nearest") if up2 else xr
    z = F.conv2d(xi, Wr, br, stride=stride, padding=pad)
    if use_emb:
        z = z + er[:, :, None, None]
    if ps:
        z = F.pixel_shuffle(z, 2)
    if act == 1:
        z = F.leaky_relu(z, slope)
    elif act == 2:
        z = F.gelu(z)
    res = torch.randn(z.shape, device="cuda", generator=g) if use_res else None
    rr = res.clone().requires_grad_(True) if use_res else None
    out_ref = z + rr if use_res else z
    gout = torch.randn(out_ref.shape, device="cuda", generator=g)
    out_ref.backward(gout)

    xo, Wo, bo = (t.clone().requires_grad_(True) for t in (x, W, b))
    eo = emb.clone().requires_grad_(True) if use_emb else None
    ro = _nhwc(res).requires_grad_(True) if use_res else None
    cfg = AG.ConvCfg(k, k, stride, pad, up2, ps, act, slope)
    xn = _nhwc(xo.detach()).requires_grad_(True)
    out = AG.conv2d(xn, Wo, bo, emb=eo, res=ro, cfg=cfg)
    assert _rel(_nchw(out), out_ref.detach()) < 1e-5
    out.backward(_nhwc(gout))
    assert _rel(_nchw(xn.grad), xr.grad) < 1e-5
    assert _rel(Wo.grad, Wr.grad) < 1e-5
    assert _rel(bo.grad, br.grad) < 1e-5
    if use_emb:
        assert _rel(eo.grad, er.grad) < 1e-5
    if use_res:
        assert _rel(_nchw(ro.grad), rr.grad) < 1e-6


@pytest.mark.parametrize("silu", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_group_norm_backward(gpu, silu, dt):
    from rdeic_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(3)
    n, c, h, w, groups = 2, 64, 9, 17, 16
    x = torch.randn((n, c, h, w), device="cuda", generator=g) * 2 + 0.5
    ga = torch.rand(c, device="cuda", generator=g) + 0.5
    be = torch.randn(c, device="cuda", generator=g) * 0.1
    xr, gr, br = (t.clone().to(dt).float().requires_grad_(True) for t in (x, ga, be))
    y = F.group_norm(xr, groups, gr, br, 1e-5)
    if silu:
        y = F.silu(y)
    gy = torch.randn(y.shape, device="cuda", generator=g)
    y.backward(gy.to(dt).float())
    xo = _nhwc(x).to(dt).requires_grad_(True)
    go, bo = ga.clone().requires_grad_(True), be.clone().requires_grad_(True)
    yo = AG.group_norm(xo, go, bo, groups, 1e-5, silu)
    yo.backward(_nhwc(gy).to(dt))
    tol = 1e-4 if dt == torch.float32 else 3e-2
    assert _rel(_nchw(yo), y.detach()) < tol
    assert _rel(_nchw(xo.grad), xr.grad) < tol
    assert _rel(go.grad, gr.grad) < tol
    assert _rel(bo.grad, br.grad) < tol


def test_layer_norm_backward(gpu):
    from rdeic_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(4)
    rows, c = 300, 320
    x = torch.randn((rows, c), device="cuda", generator=g)
    ga = torch.rand(c, device="cuda", generator=g) + 0.5
    be = torch.randn(c, device="cuda", generator=g) * 0.1
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, ga, be))
    y = F.layer_norm(xr, (c,), gr, br, 1e-5)
    gy = torch.randn(y.shape, device="cuda", generator=g)
    y.backward(gy)
    xo, go, bo = (t.clone().requires_grad_(True) for t in (x, ga, be))
    yo = AG.layer_norm(xo, go, bo)
    yo.backward(gy)
    for a, b in ((yo, y), (xo.grad, xr.grad), (go.grad, gr.grad), (bo.grad, br.grad)):
        assert _rel(a, b.detach()) < 1e-4


@pytest.mark.parametrize("dh,lk,B,L", [(64, None, 2, 96), (16, None, 2, 96), (64, 77, 2, 96),
                                       (16, None, 1, 1024), (64, 77, 1, 1024)])  # B=1: split-K dK / dV
def test_attention_backward(gpu, dh, lk, B, L):
    from rdeic_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(5)
    H = 3
    Lk = L if lk is None else lk
    q = torch.randn((B * L, H * dh), device="cuda", generator=g)
    k = torch.randn((B * Lk, H * dh), device="cuda", generator=g)
    v = torch.randn((B * Lk, H * dh), device="cuda", generator=g)
    scale = dh ** -0.5
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    qh = qr.view(B, L, H, dh).transpose(1, 2)
    kh = kr.view(B, Lk, H, dh).transpose(1, 2)
    vh = vr.view(B, Lk, H, dh).transpose(1, 2)
    o = (torch.softmax(qh @ kh.transpose(-1, -2) * scale, -1) @ vh).transpose(1, 2).reshape(B * L, H * dh)
    go = torch.randn(o.shape, device="cuda", generator=g)
    o.backward(go)
    qo, ko, vo = (t.clone().requires_grad_(True) for t in (q, k, v))
    oo = AG.attention(qo, ko, vo, B, H, scale)
    oo.backward(go)
    for a, b in ((oo, o), (qo.grad, qr.grad), (ko.grad, kr.grad), (vo.grad, vr.grad)):
        assert _rel(a, b.detach()) < 1e-4


def test_geglu_and_act_backward(gpu):
    from rdeic_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.randn((50, 2 * 40), device="cuda", generator=g)
    xr = x.clone().requires_grad_(True)
    a, gate = xr.chunk(2, dim=-1)
    y = a * F.gelu(gate)
    gy = torch.randn(y.shape, device="cuda", generator=g)
    y.backward(gy)
    xo = x.clone().requires_grad_(True)
    yo = AG.geglu(xo)
    yo.backward(gy)
    assert _rel(yo, y.detach()) < 1e-5 and _rel(xo.grad, xr.grad) < 1e-5
    for kind, fn in ((AG.SILU, F.silu), (AG.GELU, F.gelu), (AG.LEAKY, lambda t: F.leaky_relu(t, 0.01))):
        zr = x.clone().requires_grad_(True)
        fn(zr).backward(x)
        zo = x.clone().requires_grad_(True)
        AG.act(zo, kind, 0.01).backward(x)
        assert _rel(zo.grad, zr.grad) < 1e-5


def test_checkerboard_likelihood_backward(gpu):
    """CkbdAnchorFn / CkbdLikFn against oracle/train_ref.py (the compressai 1.2.4 restatement the
    golden step also uses), run with torch autograd on the GPU."""
    from oracle import train_ref
    from rdeic_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(7)
    n, c, h, w = 2, 8, 6, 10
    y = torch.randn((n, c, h, w), device="cuda", generator=g) * 3
    pa = torch.randn((n, 2 * c, h, w), device="cuda", generator=g)
    pn = torch.randn((n, 2 * c, h, w), device="cuda", generator=g)
    pa[:, :c] = pa[:, :c].abs() * 2     # scales, some below the 0.11 bound
    pn[:, :c] = pn[:, :c].abs() * 2
    noise = torch.rand((n, c, h, w), device="cuda", generator=g) - 0.5
    mask_a = torch.zeros((1, 1, h, w), device="cuda")
    mask_a[:, :, 0::2, 1::2] = 1
    mask_a[:, :, 1::2, 0::2] = 1
    mask_n = 1 - mask_a
    yr, par, pnr = (t.clone().requires_grad_(True) for t in (y, pa, pn))
    sa, ma = par.chunk(2, 1)
    sn, mn = pnr.chunk(2, 1)
    anchor = train_ref.quantize_ste(yr * mask_a - ma * mask_a) + ma * mask_a
    scales = sa * mask_a + sn * mask_n
    means = ma * mask_a + mn * mask_n
    _, lik = train_ref.gaussian_forward(yr, scales, means, True, noise=noise)
    non = train_ref.quantize_ste(yr * mask_n - mn * mask_n) + mn * mask_n
    S = torch.log(lik).sum()
    gA = torch.randn(anchor.shape, device="cuda", generator=g)
    gN = torch.randn(non.shape, device="cuda", generator=g)
    (S * -0.7 + (anchor * gA).sum() + (non * gN).sum()).backward()
    yo = _nhwc(y).requires_grad_(True)
    pao = _nhwc(pa).requires_grad_(True)
    pno = _nhwc(pn).requires_grad_(True)
    anc = AG.CkbdAnchorFn.apply(yo, pao)
    So, qSo, nono = AG.CkbdLikFn.apply(yo, pao, pno, _nhwc(noise))
    assert _rel(_nchw(anc), anchor.detach()) < 1e-6 and _rel(_nchw(nono), non.detach()) < 1e-6
    assert abs(float(So) - float(S)) < 1e-4 * abs(float(S))
    (So * -0.7 + (anc * _nhwc(gA)).sum() + (nono * _nhwc(gN)).sum()).backward()
    assert _rel(_nchw(yo.grad), yr.grad) < 1e-4
    assert _rel(_nchw(pao.grad), par.grad) < 1e-4
    assert _rel(_nchw(pno.grad), pnr.grad) < 1e-4


def test_adamw_kernel_matches_torch(gpu):
    from rdeic_amd import autograd as AG
    g = torch.Generator(device="cuda").manual_seed(8)
    p0 = torch.randn(5000, device="cuda", generator=g)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=2e-5, foreach=False)
    p, m, v = p0.clone(), torch.zeros_like(p0), torch.zeros_like(p0)
    for step in range(1, 4):
        gr = torch.randn(5000, device="cuda", generator=g)
        ref.grad = gr.clone()
        opt.step()
        AG.adamw_(p, gr, m, v, step, 2e-5)
    assert float((p - ref.detach()).abs().max()) <= 2e-7


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_pack_batch_matches_single_packs(gpu, dt):
    """rdeic_pack_batch (every trainable layer's packing in one launch) == the per-layer packers."""
    from rdeic_amd import autograd as AG, ops
    g = torch.Generator(device="cuda").manual_seed(9)
    shapes = [(320, 256, 3, 3), (64, 260, 3, 3), (1280, 320, 1, 1), (16, 8, 5, 5)]
    ws = [torch.randn(s, device="cuda", generator=g) for s in shapes]
    sp = AG.StepPacks()
    refs = []
    with sp.active():
        for w in ws:
            p = ops.ConvParams.pack(w, None, dtype=dt)
            sp.register(w, dt, 0, torch.empty_like(p.weight), p.wld, *w.shape)
            refs.append(p.weight)
            cout, cin, kh, kw = w.shape
            wld = -(-(kh * kw * cout) // 64) * 64
            ref_d = torch.empty((cin, wld), dtype=dt, device="cuda")
            ops.call("rdeic_pack_conv_weight_dgrad", w.data_ptr(), cout, cin, kh, kw, ref_d.data_ptr(), wld,
                     int(dt == torch.bfloat16), ops.stream_ptr())
            sp.register(w, dt, 1, torch.full_like(ref_d, 7.0), wld, *w.shape)
            refs.append(ref_d)
        sp.refresh()
        for w in ws:
            for mode in (0, 1):
                assert sp.lookup(w, dt, mode) is not None
    for (w, packed, *_), ref in zip(sp.jobs, refs):
        assert torch.equal(packed, ref)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_backward_keeps_forward_splitk(gpu, dt):
    """autograd runs Conv2dFn.backward on its own engine thread, whose split-K
    switches are off, so the B=1 input-gradient convs of the fine-tune step stopped splitting K.
    The backward now re-enters the forward thread's state (ops.splitk_as): under
    splitk_allowed(short_k=True) the 8x8 1280-channel dgrad conv must run split, and match torch."""
    from rdeic_amd import autograd as AG, ops
    g = torch.Generator(device="cuda").manual_seed(5)
    cin = cout = 1280
    x = torch.randn((1, cin, 8, 8), device="cuda", generator=g)
    W = torch.randn((cout, cin, 3, 3), device="cuda", generator=g) / math.sqrt(cin * 9)
    gout = torch.randn((1, cout, 8, 8), device="cuda", generator=g)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, W, None, padding=1).backward(gout)
    xn = _nhwc(x).to(dt).requires_grad_(True)
    Wo = W.clone()  # frozen fp32 master (the UNet's), packed in the compute dtype: only the input gradient
    cfg = AG.ConvCfg(3, 3, 1, 1)
    with ops.splitk_allowed(short_k=True):
        out = AG.conv2d(xn, Wo, None, cfg=cfg)
        ops.launch_count_reset()
        out.backward(_nhwc(gout).to(dt))
        torch.cuda.synchronize()
    assert ops.launch_count(ops.COUNT_SPLITK) >= 1
    assert ops.splitk_state() == (False, False)  # nothing leaked into this thread
    assert _rel(_nchw(xn.grad.float()), xr.grad) < (1e-5 if dt == torch.float32 else 2e-2)
