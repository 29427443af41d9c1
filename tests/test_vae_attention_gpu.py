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
