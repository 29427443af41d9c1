"""Parity at config 3's size (BASELINE.json configs[2]: 1024x1024 images, latent 128², y 64²,
z 16², 1,048,576 entropy-coded symbols per image), through the HIP path.

* fp32: the GPU's compressor nets + checkerboard stages + rANS/AC coders, fed the GPU's own VAE
  feature h, write the same file body as the CPU oracle (oracle/model_ref.compress, which restates
  model/compression.py:151-213 + utils/ckbd.py:76-134) fed that same h; decompressing that body
  reproduces the oracle's c_latent / guide_hint (compression.py:215-273) within fp32 tolerance.
* fp32 VAE decode at 1024^2 (latent 128^2, the mid-block AttnBlock at L = 16384): against the
  REFERENCE Decoder's output on the same latent (tests/golden/decode_1024.npz, made by
  tests/golden/make_decode1024_golden.py from the reference's modules): pixels within 1e-3 abs.
* bf16 at config 3's batch of 8: size-independent properties — the decoder decodes its own
  streams, coding is batch-invariant (solo bytes == in-batch bytes, solo latents == in-batch
  latents), and the 5-step relay decode (config 3's S) of one image alone gives its in-batch
  pixels bit for bit (split-K counts are per image, ops.SPLITK_NOMINAL_BATCH).
The images are the seeded synthetic generator's; weights are the counter-based
synthetic set at the bench's rate gain (~0.08 bpp at 512²)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
SIZE = 1024


def _imgs(n):
    from rdeic_amd.synthetic import synth_image
    return torch.from_numpy(np.stack([synth_image(SIZE, SIZE, 231 + i) for i in range(n)])).cuda()


def test_config3_fp32_bitstream_and_decompress_vs_oracle(gpu):
    from oracle import model_ref as M
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    g = W.RATE_GAIN_BPP008
    m32 = RDEIC(compute_dtype=torch.float32).init_synthetic(rate_gain=g)
    imgs = _imgs(1)
    h = m32.encode_images_nhwc(imgs)
    assert tuple(h.shape) == (1, SIZE // 8, SIZE // 8, 512)
    out = m32.preprocess_model.compress(h)
    from rdeic_amd import bitstream
    body = bitstream.pack_body(out[0]["shape"], out[0]["strings"])
    sd = M.synthetic_state_dict(rate_gain=g)
    tables = M.Tables()
    h_cpu = h.permute(0, 3, 1, 2).contiguous().cpu()
    with torch.no_grad():
        ref_body, ref_sym, _ = M.compress(sd, h_cpu, tables, coder="c")
    assert np.asarray(ref_sym).size == (SIZE // 16) ** 2 * 256  # 1,048,576 symbols
    print(f"1024² body {len(body)} B ({8.0 * len(body) / SIZE ** 2:.4f} bpp), oracle {len(ref_body)} B")
    assert body == ref_body
    c_lat, hint = m32.decompress_bodies([body])
    with torch.no_grad():
        c_ref, h_ref = M.decompress(sd, ref_body, tables, coder="c")
    for got, ref in ((c_lat, c_ref), (hint, h_ref)):
        got = got.float().permute(0, 3, 1, 2).cpu()
        err = (got - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
        assert err < 1e-4, err


def test_config3_fp32_vae_decode_vs_reference(gpu):
    import os
    from rdeic_amd import ops
    from rdeic_amd.rdeic import RDEIC
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "decode_1024.npz"))
    m32 = RDEIC(compute_dtype=torch.float32).init_synthetic()
    lat = SIZE // 8
    z = ops.fill_uniform(torch.empty(4 * lat * lat, dtype=torch.float32, device="cuda"), int(g["z_seed"]),
                         float(g["z_scale"]), 0.0).view(1, lat, lat, 4)
    with torch.no_grad():
        x = m32.decode_nhwc(z)[0].cpu()  # [1024, 1024, 3] fp32, decode_first_stage before the clamp
    errs = [(x[r:r + 64, c:c + 64] - torch.from_numpy(ref)).abs().max().item()
            for (r, c), ref in zip(g["crops"], g["crop_pixels"])]
    print(f"1024^2 decode vs reference: crop max abs err {max(errs):.2e}; "
          f"row-mean err {np.abs(x.double().mean(1).numpy() - g['row_mean']).max():.2e}")
    assert max(errs) < 1e-3  # north-star bar: decoded pixels within 1e-3 abs (fp32)
    assert np.abs(x.double().mean(1).numpy() - g["row_mean"]).max() < 1e-4
    assert np.abs(x.double().mean(0).numpy() - g["col_mean"]).max() < 1e-4
    assert abs(x.double().sum().item() - float(g["total"])) <= 1e-5 * x.numel()


def test_config3_bf16_batch8_self_consistent_and_batch_invariant(gpu):
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, sampler_noise
    m16 = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
    B = 8
    imgs = _imgs(B)
    bodies = m16.compress_images(imgs)
    solo = m16.compress_images(imgs[1:2])
    assert solo[0] == bodies[1]
    c_b, h_b = m16.decompress_bodies(bodies)
    c_s, h_s = m16.decompress_bodies(bodies[1:2])
    assert torch.equal(c_b[1:2], c_s) and torch.equal(h_b[1:2], h_s)
    ctx = synth_context().cuda()
    _, noise = sampler_noise((B, 4, SIZE // 8, SIZE // 8), 231)
    out, bodies2 = m16.codec_images(imgs, ctx, noise, steps=5)
    assert bodies2 == bodies
    assert tuple(out.shape) == (B, SIZE, SIZE, 3) and out.dtype == torch.uint8
    out1, _ = m16.codec_images(imgs[1:2], ctx, noise[1:2], steps=5)
    assert torch.equal(out1[0], out[1])  # one image alone decodes to its in-batch pixels
    print("config-3 bpp:", [round(8.0 * len(b) / SIZE ** 2, 4) for b in bodies])


def test_config3_fp32_noise_estimator_vs_reference(gpu):
    """Config 3's relay denoiser in fp32 at latent 128^2 (the UNet's first-level self-attention at
    L = 16384, d = 64): one NoiseEstimator call (control + SD-2.1 UNet, model/rdeic.py:174-212) at t = 151
    against the REFERENCE's own modules on the same inputs (tests/golden/eps_1024.npz, made by
    tests/golden/make_eps1024_golden.py): eps within 1e-3 relative to its largest magnitude."""
    import os
    from rdeic_amd import ops
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "eps_1024.npz"))
    m32 = RDEIC(compute_dtype=torch.float32).init_synthetic()
    lat = SIZE // 8

    def field(ch, seed, scale):
        return ops.fill_uniform(torch.empty(ch * lat * lat, dtype=torch.float32, device="cuda"), int(seed),
                                float(scale), 0.0).view(1, lat, lat, ch)

    x = field(4, g["x_seed"], g["x_scale"])
    hint = field(256, g["hint_seed"], g["hint_scale"])
    t = torch.full((1,), int(g["t"]), dtype=torch.long, device="cuda")
    with torch.no_grad():
        e = m32.eps_nhwc(x, t, hint, synth_context().cuda())[0].float().cpu().numpy()
    ref = g["eps"]
    rel = np.abs(e - ref).max() / np.abs(ref).max()
    print(f"1024^2 eps vs reference: max abs err {np.abs(e - ref).max():.2e}, rel {rel:.2e}, "
          f"mean abs err {np.abs(e - ref).mean():.2e}")
    assert rel < 1e-3
