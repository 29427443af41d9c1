"""End-to-end parity on the MI355X against golden fixtures produced by the reference's own
modules (tests/golden/make_golden.py) at 128x128, batch of 2 images run as ONE batch.

fp32 parity mode: every stage must match the reference within fp32 tolerance; the integer
bitstream must be byte-identical (modulo the documented near-tie hazard of round(y - mu)).
bf16 perf mode: encoder/decoder self-consistency and closeness to the fp32 reconstruction."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "e2e_128.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.fixture(scope="module")
def model32(gpu):
    from rdeic_amd.rdeic import RDEIC
    return RDEIC(compute_dtype=torch.float32).init_synthetic()


def _nhwc(a):
    return torch.from_numpy(a).permute(0, 2, 3, 1).contiguous().cuda()


def _nchw_np(t):
    return t.float().permute(0, 3, 1, 2).cpu().numpy()


def _close(a, b, rtol, atol_rel):
    scale = max(np.abs(b).max(), 1e-6)
    err = np.abs(a - b).max()
    assert err <= atol_rel * scale + rtol * 0, f"max err {err:.3e} vs scale {scale:.3e}"
    return err / scale


def test_weights_match_oracle_generator(model32):
    from oracle import weights_cpu
    from rdeic_amd import weights as W
    for name in ("model.diffusion_model.input_blocks.1.0.in_layers.2.weight",
                 "control_model.control_model.input_blocks.0.0.weight",
                 "first_stage_model.decoder.up.0.block.2.norm1.weight",
                 "preprocess_model.quantize.embedding.weight"):
        t = model32.store.get(name)
        sc, off = W.init_spec(name, tuple(t.shape))
        ref = weights_cpu.fill_uniform(t.numel(), W.param_seed(name), sc, off)
        assert np.array_equal(t.cpu().numpy().reshape(-1), ref), name


def test_encoder_and_latents_fp32(model32, gold):
    imgs = torch.from_numpy(np.stack([gold["img0_in"], gold["img1_in"]])).cuda()
    h = model32.encode_images_nhwc(imgs)
    for i in range(2):
        c = gold[f"img{i}_vae_c"] * 0.18215
        e = _close(_nchw_np(h[i:i + 1]), c, 0, 2e-4)
        print(f"img{i} h rel err {e:.2e}")
    comp = model32.preprocess_model
    y = comp._seq(comp.g_a, h)
    z = comp._seq(comp.hyper_enc, y)
    for i in range(2):
        _close(_nchw_np(y[i:i + 1]), gold[f"img{i}_y"], 0, 2e-4)
        _close(_nchw_np(z[i:i + 1]), gold[f"img{i}_z"], 0, 2e-4)
    _, idx = comp.vq_quant(z)
    for i in range(2):
        assert np.array_equal(idx[i].cpu().numpy(), gold[f"img{i}_z_idx"][0])


def test_bitstream_fp32(model32, gold):
    """Compressed files vs the reference's (symbols and bytes)."""
    imgs = torch.from_numpy(np.stack([gold["img0_in"], gold["img1_in"]])).cuda()
    bodies = model32.compress_images(imgs)
    exact = 0
    for i in range(2):
        if bodies[i] == gold[f"img{i}_file"].tobytes():
            exact += 1
        else:
            # tolerate only the documented near-tie hazard: decode our stream and compare symbols
            from rdeic_amd import bitstream, coders
            strings, shape = bitstream.unpack_body(bodies[i])
            assert strings[1][0] == gold[f"img{i}_z_string"].tobytes()
            dec = coders.RansDecoder(strings[0][0])
            sym = dec.decode_stream(gold[f"img{i}_indexes"], model32.preprocess_model.tables)
            mism = int((sym != gold[f"img{i}_symbols"]).sum())
            assert mism <= 2, f"{mism} symbols differ"
    print(f"byte-exact files: {exact}/2")


def test_decompress_sample_decode_fp32(model32, gold):
    bodies = [gold["img0_file"].tobytes(), gold["img1_file"].tobytes()]
    c_lat, hint = model32.decompress_bodies(bodies)
    for i in range(2):
        _close(_nchw_np(c_lat[i:i + 1]), gold[f"img{i}_c_latent"], 0, 1e-4)
        _close(_nchw_np(hint[i:i + 1]), gold[f"img{i}_guide_hint"], 0, 1e-4)
    ctx = torch.from_numpy(gold["context"]).cuda()
    # relay sampling from the reference's own decompressed latents + noise
    c_ref = torch.cat([_nhwc(gold["img0_c_latent"]), _nhwc(gold["img1_c_latent"])])
    h_ref = torch.cat([_nhwc(gold["img0_guide_hint"]), _nhwc(gold["img1_guide_hint"])])
    noise = torch.cat([_nhwc(gold["img0_noise"]), _nhwc(gold["img1_noise"])])
    t = torch.full((2,), 299, dtype=torch.long, device="cuda")
    x_T = model32.q_sample_nhwc(c_ref, t, noise)
    for i in range(2):
        _close(_nchw_np(x_T[i:i + 1]), gold[f"img{i}_x_T"], 0, 1e-6)
    e = model32.eps_nhwc(x_T, torch.full((2,), 151, dtype=torch.long, device="cuda"), h_ref, ctx)
    for i in range(2):
        err = _close(_nchw_np(e[i:i + 1]), gold[f"img{i}_eps"][0], 0, 1e-3)
        print(f"eps rel err {err:.2e}")
    from rdeic_amd.ddim_sampler_relay import DDIMSampler
    z = DDIMSampler(model32).sample_nhwc(2, x_T, h_ref, ctx)
    for i in range(2):
        _close(_nchw_np(z[i:i + 1]), gold[f"img{i}_samples"], 0, 1e-3)
    x = model32.decode_nhwc(z)
    for i in range(2):
        err = np.abs(_nchw_np(x[i:i + 1]) - gold[f"img{i}_x_dec"]).max()
        print(f"decoded pixels max abs err {err:.2e}")
        assert err < 1e-3  # north-star bar: decoded pixels within 1e-3 abs (fp32)
    u8 = model32.to_image_u8(x).cpu().numpy()
    for i in range(2):
        d = np.abs(u8[i].astype(int) - gold[f"img{i}_image_out"][0].astype(int))
        assert d.max() <= 1 and (d > 0).mean() < 0.01


def test_codec_bf16_self_consistent(gpu, gold, model32):
    """bf16 perf mode: compress/decompress agree exactly with each other (batch-invariant entropy
    model) and the reconstruction stays close to the fp32 parity path."""
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd import bitstream, coders
    m16 = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    imgs = torch.from_numpy(np.stack([gold["img0_in"], gold["img1_in"]])).cuda()
    ctx = torch.from_numpy(gold["context"]).cuda()
    noise = torch.cat([torch.from_numpy(gold["img0_noise"]), torch.from_numpy(gold["img1_noise"])])
    out16, bodies = m16.codec_images(imgs, ctx, noise, steps=2)
    # batch invariance: coding image 1 alone gives the same bytes as inside the batch
    solo = m16.compress_images(imgs[1:2])
    assert solo[0] == bodies[1]
    c_b, _ = m16.decompress_bodies(bodies)
    c_s, _ = m16.decompress_bodies(bodies[1:])
    assert torch.equal(c_b[1:2], c_s)
    out32, _ = model32.codec_images(imgs, ctx, noise, steps=2)
    diff = (out16.float() - out32.float()).abs()
    print(f"bf16 vs fp32 reconstruction: mean |d| {diff.mean().item():.2f} / 255, max {diff.max().item():.0f}")
    assert diff.mean().item() < 8.0


def test_low_rate_bitstream_vs_oracle(gpu, gold):
    """The bench's ~0.08 bpp synthetic regime (weights.RATE_GAIN_BPP008): fp32 GPU files equal
    the CPU oracle's (same weight spec, C rANS twin) and the bf16 path decodes its own streams."""
    from oracle import model_ref as M
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    g = W.RATE_GAIN_BPP008
    m32 = RDEIC(compute_dtype=torch.float32).init_synthetic(rate_gain=g)
    imgs = torch.from_numpy(np.stack([gold["img0_in"], gold["img1_in"]])).cuda()
    bodies = m32.compress_images(imgs)
    sd = M.synthetic_state_dict(rate_gain=g)
    tables = M.Tables()
    with torch.no_grad():
        for i in range(2):
            x = torch.tensor(gold[f"img{i}_in"][None] / 255.0, dtype=torch.float32).permute(0, 3, 1, 2).contiguous()
            body, _, _ = M.compress(sd, M.vae_encode_hc(sd, x * 2 - 1) * 0.18215, tables, coder="c")
            assert bodies[i] == body, f"image {i}: {len(bodies[i])} vs oracle {len(body)} bytes"
    print("low-rate bpp:", [8.0 * len(b) / (128 * 128) for b in bodies])
    m16 = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=g)
    b16 = m16.compress_images(imgs)
    c_b, h_b = m16.decompress_bodies(b16)
    solo = m16.compress_images(imgs[:1])
    assert solo[0] == b16[0]
    c_s, _ = m16.decompress_bodies(b16[:1])
    assert torch.equal(c_b[:1], c_s)
