"""Parity at config 2's full size (BASELINE.json configs[1]: 512x512 images, latent 64², y 32²,
z 8², 262,144 entropy-coded symbols per image; batch 16 in bf16), through the HIP path.

* fp32, one 512² image, against the CPU oracle (oracle/model_ref.py):
  - the VAE feature h (Encoder.forward_hc, model.py:551-577) within fp32 tolerance;
  - the file body (inference.py:55-60 -> compression.py:151-213 + utils/ckbd.py:76-134 +
    utils/utils.py:57-80): byte-identical to oracle.compress fed the GPU's h (integer path,
    no tolerance), and to the oracle's own end-to-end body up to the documented round(y - mu)
    near-tie hazard (<= 2 symbols);
  - decompress (compression.py:215-273), 2-step relay DDIM (ddim_sampler_relay.py:23-231) and VAE
    decode (model.py:653-686) from that body: decoded pixels within 1e-3 abs of the oracle's
    (the north star's fp32 bar), and the uint8 output (truncating cast, inference.py:85-87).
* bf16, the bench's batch of 16 (config 2 exactly): the decoder decodes its own streams, coding
  is batch-invariant (solo == in-batch bytes and latents), the 2-step relay latent is finite, the
  codec loop returns the same bodies, and the bpp sits at config 2's ~0.08.
Weights: the counter-based synthetic set at the bench's rate gain; images: the seeded generator."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
SIZE = 512


def _imgs(seeds):
    from rdeic_amd.synthetic import synth_image
    return torch.from_numpy(np.stack([synth_image(SIZE, SIZE, s) for s in seeds])).cuda()


def _nchw(t):
    return t.float().permute(0, 3, 1, 2).contiguous().cpu()


def test_config2_fp32_image_vs_oracle(gpu):
    from oracle import model_ref as M
    from rdeic_amd import bitstream, coders
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import sampler_noise, synth_context
    g = W.RATE_GAIN_BPP008
    m32 = RDEIC(compute_dtype=torch.float32).init_synthetic(rate_gain=g)
    img = _imgs([231])
    sd = M.synthetic_state_dict(rate_gain=g)
    tables = M.Tables()
    torch.set_num_threads(16)
    with torch.no_grad():
        # encoder
        h = m32.encode_images_nhwc(img)
        x = torch.tensor(img.cpu().numpy() / 255.0, dtype=torch.float32).permute(0, 3, 1, 2).contiguous()
        h_ref = M.vae_encode_hc(sd, x * 2 - 1) * 0.18215
        err = ((_nchw(h) - h_ref).abs().max() / h_ref.abs().max()).item()
        print(f"512² h rel err {err:.2e}")
        assert err < 2e-4
        # file body: the integer path is exact from the same h
        out = m32.preprocess_model.compress(h)
        body = bitstream.pack_body(out[0]["shape"], out[0]["strings"])
        body_from_h, _, _ = M.compress(sd, _nchw(h), tables, coder="c")
        assert body == body_from_h, f"{len(body)} B vs oracle-from-GPU-h {len(body_from_h)} B"
        ref_body, ref_sym, ref_idx = M.compress(sd, h_ref, tables, coder="c")
        assert np.asarray(ref_sym).size == (SIZE // 16) ** 2 * 256  # 262,144 symbols
        print(f"512² body {len(body)} B ({8.0 * len(body) / SIZE ** 2:.4f} bpp); oracle end-to-end "
              f"{len(ref_body)} B, byte-identical: {body == ref_body}")
        if body != ref_body:  # only the near-tie hazard of round(y - mu) may separate them
            strings, _ = bitstream.unpack_body(body)
            rs, _ = bitstream.unpack_body(ref_body)
            assert strings[1][0] == rs[1][0]  # hyper-latent (VQ index) string
            sym = coders.RansDecoder(strings[0][0]).decode_stream(np.asarray(ref_idx), m32.preprocess_model.tables)
            mism = int((np.asarray(sym) != np.asarray(ref_sym)).sum())
            assert mism <= 2, f"{mism} symbols differ"
        # decompress -> 2-step relay DDIM -> VAE decode, both sides from the oracle's own body
        c_lat, hint = m32.decompress_bodies([ref_body])
        c_ref, hint_ref = M.decompress(sd, ref_body, tables, coder="c")
        for got, ref in ((c_lat, c_ref), (hint, hint_ref)):
            e = ((_nchw(got) - ref).abs().max() / ref.abs().max()).item()
            assert e < 1e-4, e
        ctx = synth_context()
        _, noise = sampler_noise((1, 4, SIZE // 8, SIZE // 8), 231)
        z = m32.relay_sample_nhwc(c_lat, hint, ctx.cuda(), noise.permute(0, 2, 3, 1).contiguous().cuda(), steps=2)
        xdec = m32.decode_nhwc(z)
        sched = M.schedule()
        t = torch.full((1,), 299, dtype=torch.long)
        x_t = sched["sqrt_alphas_cumprod"][t].view(-1, 1, 1, 1) * c_ref + \
            sched["sqrt_one_minus_alphas_cumprod"][t].view(-1, 1, 1, 1) * noise
        z_ref = M.ddim_relay(sd, x_t, hint_ref, ctx, 2, sched)
        e = ((_nchw(z) - z_ref).abs().max() / z_ref.abs().max()).item()
        print(f"512² relay latent rel err {e:.2e}")
        assert e < 1e-3
        x_ref = M.vae_decode(sd, z_ref / 0.18215)
        err = (_nchw(xdec) - x_ref).abs().max().item()
        print(f"512² decoded pixels max abs err {err:.2e}")
        assert err < 1e-3  # north-star bar: decoded pixels within 1e-3 abs (fp32)
        u8 = m32.to_image_u8(xdec).cpu().numpy()[0]
        u8_ref = (((x_ref + 1) / 2).clamp(0, 1).permute(0, 2, 3, 1) * 255).numpy().clip(0, 255).astype(np.uint8)[0]
        d = np.abs(u8.astype(int) - u8_ref.astype(int))
        assert d.max() <= 1 and (d > 0).mean() < 0.01


def test_config2_bf16_batch16(gpu):
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context
    m16 = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
    seeds = list(range(231, 247))
    imgs = _imgs(seeds)
    with torch.no_grad():
        bodies = m16.compress_images(imgs)
        assert len(bodies) == 16
        solo = m16.compress_images(imgs[5:6])
        assert solo[0] == bodies[5]
        c_b, h_b = m16.decompress_bodies(bodies)
        c_s, h_s = m16.decompress_bodies(bodies[5:6])
        assert torch.equal(c_b[5:6], c_s) and torch.equal(h_b[5:6], h_s)
        ctx = synth_context().cuda()
        noise = torch.cat([relay_noise((1, 4, SIZE // 8, SIZE // 8), s, 2)[0] for s in seeds])
        z = m16.relay_sample_nhwc(c_b, h_b, ctx, noise.permute(0, 2, 3, 1).contiguous().cuda(), steps=2)
        assert tuple(z.shape) == (16, SIZE // 8, SIZE // 8, 4) and bool(torch.isfinite(z).all())
        out, bodies2 = m16.codec_images(imgs, ctx, noise, steps=2)
        assert bodies2 == bodies
        assert tuple(out.shape) == (16, SIZE, SIZE, 3) and out.dtype == torch.uint8
    bpp = [8.0 * len(b) / SIZE ** 2 for b in bodies]
    print(f"config-2 bf16 mean bpp {np.mean(bpp):.4f} (min {min(bpp):.4f}, max {max(bpp):.4f})")
    assert 0.04 < np.mean(bpp) < 0.12
