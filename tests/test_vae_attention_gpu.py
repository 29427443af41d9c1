"""The VAE AttnBlock's single-head d=512 attention (model.py:181-205) with a bounded score
buffer: chunked by images and by query rows it must give exactly the unchunked result (same k
order per output row), and match a torch fp32 reference of softmax(q k^T * C^-1/2) v."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_single_head_attention_chunked_is_exact(gpu, dtype):
    from rdeic_amd import ops
    B, L, C = 3, 1024, 512
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(B * L, C, device="cuda", generator=g).to(dtype) for _ in range(3))
    scale = C ** -0.5
    full = torch.empty(B * L, C, dtype=dtype, device="cuda")
    prev = ops.SCORE_BUDGET_BYTES
    try:
        ops.SCORE_BUDGET_BYTES = 1 << 40  # everything in one chunk
        ops.attention_single_head_materialized(q, k, v, full, batch=B, length=L, dim=C, scale=scale)
        for budget in (2 * L * L * 4, L * L * 4 // 4 + 1, 64 * L * 4):  # 2 images / 1/4 image / 64 rows
            ops.SCORE_BUDGET_BYTES = budget
            part = torch.empty_like(full)
            ops.attention_single_head_materialized(q, k, v, part, batch=B, length=L, dim=C, scale=scale)
            assert torch.equal(part, full), budget
    finally:
        ops.SCORE_BUDGET_BYTES = prev
    ref = torch.softmax((q.float().view(B, L, C) @ k.float().view(B, L, C).transpose(1, 2)) * scale, -1) \
        @ v.float().view(B, L, C)
    tol = 2e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(full.float().view(B, L, C), ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("B,L,spread", [(2, 1024, 1.0), (1, 4096, 1.0), (2, 256, 6.0), (1, 96, 1.0),
                                        (1, 16384, 1.0)])  # 16384: config 3's 1024^2 mid-block
def test_flash_d512_matches_fp32_reference(gpu, B, L, spread):
    """The flash kernel (rdeic_attention, dh = 512, bf16): no score buffer; against torch fp32 on the
    same bf16 inputs, on the AttnBlock's [B*L, 3C] qkv layout (row stride 3C). spread > 1 gives
    large logits so the deferred-max rescale path runs; L = 96 has a partial 64-query block."""
    from rdeic_amd import ops
    C = 512
    g = torch.Generator(device="cuda").manual_seed(L)
    qkv = (torch.randn(B * L, 3 * C, device="cuda", generator=g) * spread).to(torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    scale = C ** -0.5
    out = torch.empty(B * L, C, dtype=torch.bfloat16, device="cuda")
    ops.attention(q, k, v, out, batch=B, heads=1, lq=L, lk=L, dh=C, scale=scale)
    torch.cuda.synchronize()
    qf, kf, vf = (t.float().reshape(B, L, C) for t in (q, k, v))
    ref = torch.softmax((qf @ kf.transpose(1, 2)) * scale, -1) @ vf
    err = (out.float().view(B, L, C) - ref).abs()
    # bf16 probabilities (P) and bf16 output: ~1e-2 relative to the output scale
    assert err.max().item() < 2e-2 * max(1.0, ref.abs().max().item()), err.max().item()
    assert err.mean().item() < 2e-3 * max(1.0, ref.abs().max().item()), err.mean().item()
    if spread == 1.0 and L % 64 == 0 and L <= 4096:
        mat = torch.empty_like(out)
        ops.attention_single_head_materialized(q, k, v, mat, batch=B, length=L, dim=C, scale=scale)
        assert (mat.float() - out.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("dh,heads,B,L,reps", [(512, 1, 8, 16384, 24), (64, 5, 8, 16384, 24), (64, 5, 16, 4096, 24)])
def test_flash_kernels_run_to_run_deterministic(gpu, dh, heads, B, L, reps):
    """Repeated launches on the same inputs give the same bits (config 3's 1024^2 shapes). The asm
    transposed V reads of attn512 / attn64 are ordered after their counted lgkmcnt waits only by
    data dependence (attention.hip tie()); without it the MFMA could read a VGPR before its LDS
    data arrived: 6-8 of 59 repeats differed at B=8, L=16384 (tools/probe/attn512_repeat.py)."""
    from rdeic_amd import ops
    C = heads * dh
    g = torch.Generator(device="cuda").manual_seed(L + dh)
    qkv = torch.randn(B * L, 3 * C, device="cuda", generator=g).to(torch.bfloat16)
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    ref = torch.empty(B * L, C, dtype=torch.bfloat16, device="cuda")
    ops.attention(q, k, v, ref, batch=B, heads=heads, lq=L, lk=L, dh=dh, scale=dh ** -0.5)
    bad = 0
    for _ in range(reps):
        o = torch.empty_like(ref)
        ops.attention(q, k, v, o, batch=B, heads=heads, lq=L, lk=L, dh=dh, scale=dh ** -0.5)
        bad += int(not torch.equal(o, ref))
    assert bad == 0, f"{bad}/{reps} repeats differ"
