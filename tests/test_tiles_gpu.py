"""Every conv tile id gives bit-identical results on every layer-shape class of the path.

The encoder and decoder entropy models must compute identical mu / sigma (SURVEY Appendix A,
hazard 8), and the per-shape tile table (rdeic_amd/conv_tiles.json) may pick any tile. This runs a
small bf16 codec (VAE encoder, entropy nets, 20 checkerboard stages, relay UNet + control, VAE
decoder) with ops.conv2d wrapped: at the first call of each distinct layer shape, the same conv is
re-run with every tile id (register tiles 0-10, LDS-DMA tiles 21-38) and with the built-in
heuristic, and each result must equal the table's output bit for bit — and so must the GroupNorm
statistics fused into the epilogue of the convs that produce them (or computed by the stand-alone
fallback where a tile cannot fuse them)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_every_tile_bit_identical_on_every_layer_shape(gpu):
    from rdeic_amd import ops
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image

    orig = ops.conv2d
    seen, checked, mismatches, stats_checked = set(), [], [], []

    def shape_key(x, p, kw):
        x2 = kw.get("x2")
        return (tuple(x.shape), None if x2 is None else x2.shape[3], p.cout, p.kh, p.kw, p.stride,
                bool(kw.get("up2")), bool(kw.get("pixel_shuffle")), bool(kw.get("geglu")), kw.get("gn") is not None,
                bool(kw.get("stats")), kw.get("stats_hw"),
                kw.get("res") is not None, kw.get("emb") is not None, kw.get("act", 0), bool(kw.get("out_f32")))

    def wrapped(x, p, **kw):
        key = shape_key(x, p, kw)
        if x.dtype != torch.bfloat16 or key in seen:
            return orig(x, p, **kw)
        seen.add(key)
        # the residual may alias the output (in-place accumulation): keep a copy for the re-runs
        kw_rerun = {k: v for k, v in kw.items() if k != "out"}
        if kw.get("res") is not None:
            kw_rerun["res"] = kw["res"].clone()
        out = orig(x, p, **kw)
        ref = out.clone()
        ref_part = getattr(out, "_rdeic_gn_part", (None,))[0]
        if ref_part is not None:
            ref_part = ref_part.clone()
            stats_checked.append(key)
        for t in (-1,) + ops.ALL_TILES:
            ops.FORCE_TILE = t
            try:
                got = orig(x, p, **kw_rerun)
            finally:
                ops.FORCE_TILE = None
            if not torch.equal(got, ref):
                mismatches.append((key, t, (got.float() - ref.float()).abs().max().item()))
            # fused GroupNorm statistics: canonical order, identical for every tile (or fallback)
            # (header word 0 = rows per partial, words 1-3 unused padding, then the sums)
            gp = None if ref_part is None else got._rdeic_gn_part[0]
            if ref_part is not None and not (torch.equal(gp[4:], ref_part[4:]) and torch.equal(gp[:1], ref_part[:1])):
                mismatches.append((key, t, "gn statistics"))
        checked.append(key)
        return out

    ops.conv2d = wrapped
    try:
        m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
        m.preprocess_model.update(force=True)
        m.use_plans = False  # every conv through ops.conv2d
        B, S = 2, 128
        imgs = torch.from_numpy(np.stack([synth_image(S, S, 700 + i) for i in range(B)])).cuda()
        noise = torch.cat([relay_noise((1, 4, S // 8, S // 8), 700 + i, 2)[0] for i in range(B)])
        out, bodies = m.codec_images(imgs, synth_context().cuda(), noise, steps=2)
        torch.cuda.synchronize()
    finally:
        ops.conv2d = orig
    assert out.shape == (B, S, S, 3) and all(len(b) > 16 for b in bodies)
    assert len(checked) > 60, len(checked)
    assert len(stats_checked) > 10, len(stats_checked)
    assert not mismatches, mismatches[:10]
