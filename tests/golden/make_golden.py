"""Generate golden fixtures by running the REFERENCE's own modules (read-only, /root/reference)
on seeded synthetic inputs with the synthetic weights of rdeic_amd/weights.py.

Run in the development container only (the reference does not exist on the GPU box):
    python -m tests.golden.make_golden
Outputs (small, committed): tests/golden/e2e_128.npz, tests/golden/param_shapes.json.

The pipeline mirrors inference.process (inference.py:22-91) at 128x128, 2-step relay DDIM:
  x = u8/255 -> Encoder.forward_hc(x*2-1) (autoencoder.py:91-95) -> h = c*0.18215
  -> Compression.compress(h) -> bytes -> Compression.decompress -> (c_latent, guide_hint)
  -> q_sample(c_latent, 299, noise) -> DDIMSampler.sample(S=2) with NoiseEstimator.forward
  -> post_quant_conv(z / 0.18215) -> Decoder -> ((x+1)/2).clamp(0,1)*255 -> uint8
compressai / torchac pieces come from oracle/coders_ref.py (see tests/golden/refload.py).
"""
from __future__ import annotations

import json
import math
import os
import struct
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import weights_cpu  # noqa: E402
from rdeic_amd import weights as W  # noqa: E402
from tests.golden import refload  # noqa: E402
from tests.golden.synth import CONFIG, synth_image, synth_context, sampler_noise  # noqa: E402


def fill_module(module: torch.nn.Module, prefix: str):
    sd = module.state_dict()
    new = {}
    for k, v in sd.items():
        full = prefix + k
        if W.is_param(full) and v.is_floating_point():
            scale, offset = W.init_spec(full, tuple(v.shape))
            arr = weights_cpu.fill_uniform(v.numel(), W.param_seed(full), scale, offset)
            new[k] = torch.from_numpy(arr).view(v.shape)
        else:
            new[k] = v
    module.load_state_dict(new, strict=True)


def build_reference():
    R = refload.load()
    cfg = CONFIG
    unet = R.UNetModel(**cfg["unet"]).eval()
    ne = R.NoiseEstimator(**cfg["control"]).eval()
    enc = R.Encoder(**cfg["ddconfig"]).eval()
    dec = R.Decoder(**cfg["ddconfig"]).eval()
    quant_conv = torch.nn.Conv2d(8, 8, 1)
    post_quant_conv = torch.nn.Conv2d(4, 4, 1)
    comp = R.Compression(**cfg["compression"]).eval()
    mods = [(unet, "model.diffusion_model."), (ne, "control_model."), (enc, "first_stage_model.encoder."),
            (dec, "first_stage_model.decoder."), (quant_conv, "first_stage_model.quant_conv."),
            (post_quant_conv, "first_stage_model.post_quant_conv."), (comp, "preprocess_model.")]
    t = time.time()
    for m, p in mods:
        fill_module(m, p)
    print(f"weights filled in {time.time() - t:.1f}s")
    shapes = {}
    for m, p in mods:
        for k, v in m.state_dict().items():
            shapes[p + k] = list(v.shape)
    return R, unet, ne, enc, dec, post_quant_conv, comp, shapes


def schedule(R):
    betas = R.util.make_beta_schedule("linear", 1000, linear_start=0.00085, linear_end=0.0120)
    alphas_cumprod = np.cumprod(1.0 - betas, axis=0)
    alphas_cumprod_prev = np.append(1.0, alphas_cumprod[:-1])
    f32 = lambda a: torch.tensor(a, dtype=torch.float32)  # noqa: E731
    return dict(betas=f32(betas), alphas_cumprod=f32(alphas_cumprod), alphas_cumprod_prev=f32(alphas_cumprod_prev),
                sqrt_alphas_cumprod=f32(np.sqrt(alphas_cumprod)),
                sqrt_one_minus_alphas_cumprod=f32(np.sqrt(1.0 - alphas_cumprod)))


class RecordingEncoder:
    """Wraps the restated BufferedRansEncoder to record the reference's symbol / index lists."""
    last = None

    def __init__(self):
        from oracle.coders_ref import RansEncoderRef
        self.inner = RansEncoderRef()
        RecordingEncoder.last = self

    def encode_with_indexes(self, symbols, indexes, cdfs, sizes, offsets):
        self.symbols, self.indexes = list(symbols), list(indexes)
        self.inner.encode_with_indexes(symbols, indexes, cdfs, sizes, offsets)

    def flush(self):
        return self.inner.flush()


def run_image(R, unet, ne, enc, dec, pqc, comp, img_u8, context, noise_pair, sched, steps):
    import model.compression as mc
    mc.BufferedRansEncoder = RecordingEncoder
    out = {}
    with torch.no_grad():
        x = torch.tensor(np.stack([img_u8]) / 255.0, dtype=torch.float32).permute(0, 3, 1, 2).contiguous()
        H, W_ = x.shape[-2:]
        _, c = enc.forward_hc(x * 2 - 1)
        h = c * CONFIG["scale_factor"]
        out["vae_c"] = c.numpy()
        # capture intermediates of the compressor
        y = comp.encoder(h)
        z = comp.hyper_enc(y)
        out["y"], out["z"] = y.numpy(), z.numpy()
        res = comp.compress(h)
        rec = RecordingEncoder.last
        out["symbols"] = np.asarray(rec.symbols, dtype=np.int32)
        out["indexes"] = np.asarray(rec.indexes, dtype=np.int32)
        y_str, z_str = res["strings"][0][0], res["strings"][1][0]
        zh, zw = [int(v) for v in res["shape"]]
        body = struct.pack(">3I", zh, zw, 2) + struct.pack(">I", len(y_str)) + y_str + struct.pack(">I", len(z_str)) + z_str
        out["y_string"] = np.frombuffer(y_str, dtype=np.uint8)
        out["z_string"] = np.frombuffer(z_str, dtype=np.uint8)
        out["file"] = np.frombuffer(body, dtype=np.uint8)
        out["bpp"] = np.float64(len(body) * 8 / (H * W_))
        _, idx = comp.quantize.quant(z)
        out["z_idx"] = idx.numpy().astype(np.int32)
        c_latent, guide_hint = comp.decompress([[y_str], [z_str]], (zh, zw))
        out["c_latent"], out["guide_hint"] = c_latent.numpy(), guide_hint.numpy()
        # relay sampling (inference.py:63-79), noise from the host generator
        _, noise = noise_pair
        t = torch.ones((1,)).long() * CONFIG["used_timesteps"] - 1
        x_T = (sched["sqrt_alphas_cumprod"][t].view(-1, 1, 1, 1) * c_latent +
               sched["sqrt_one_minus_alphas_cumprod"][t].view(-1, 1, 1, 1) * noise)
        out["noise"], out["x_T"] = noise.numpy(), x_T.numpy()

        class M:  # the attributes DDIMSampler / p_sample_ddim read from RDEIC
            pass
        m = M()
        m.used_timesteps = CONFIG["used_timesteps"]
        m.device = torch.device("cpu")
        m.parameterization = "eps"
        for k, v in sched.items():
            setattr(m, k, v)
        eps_list = []

        def apply_model(xn, tt, cond):
            e = ne(x=xn, guide_hint=cond["guide_hint"], timesteps=tt, context=torch.cat(cond["c_crossattn"], 1),
                   base_model=unet)
            eps_list.append((int(tt[0]), e.numpy()))
            return e
        m.apply_model = apply_model
        R.DDIMSampler.register_buffer = lambda self, name, attr: setattr(self, name, attr)
        sampler = R.DDIMSampler(m)
        cond = {"c_latent": [c_latent], "c_crossattn": [context], "guide_hint": guide_hint}
        samples, _ = sampler.sample(S=steps, batch_size=1, shape=(4, H // 8, W_ // 8), conditioning=cond,
                                    unconditional_conditioning=None, unconditional_guidance_scale=1.0, x_T=x_T, eta=0,
                                    verbose=False)
        out["eps_t"] = np.asarray([t_ for t_, _ in eps_list], dtype=np.int64)
        out["eps"] = np.stack([e for _, e in eps_list])
        out["samples"] = samples.numpy()
        z_dec = pqc(samples / CONFIG["scale_factor"])
        xs = dec(z_dec)
        out["x_dec"] = xs.numpy()
        xs = ((xs + 1) / 2).clamp(0, 1)
        out["image_out"] = (xs.permute(0, 2, 3, 1) * 255).numpy().clip(0, 255).astype(np.uint8)
    return out


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    R, unet, ne, enc, dec, pqc, comp, shapes = build_reference()
    with open(os.path.join(HERE, "param_shapes.json"), "w") as f:
        json.dump(shapes, f)
    from utils.func import get_scale_table
    comp.gaussian_conditional.update_scale_table(get_scale_table(), force=True)
    sched = schedule(R)
    ctx = synth_context()
    fixtures = {"context": ctx.numpy(), "scale_table": get_scale_table().numpy(),
                "quantized_cdf": comp.gaussian_conditional.quantized_cdf.numpy(),
                "cdf_length": comp.gaussian_conditional.cdf_length.numpy(),
                "offset": comp.gaussian_conditional.offset.numpy()}
    for k, v in sched.items():
        fixtures["sched_" + k] = v.numpy()
    for i, seed in enumerate((231, 232)):
        img = synth_image(128, 128, seed)
        t0 = time.time()
        res = run_image(R, unet, ne, enc, dec, pqc, comp, img, ctx, sampler_noise((1, 4, 16, 16), seed), sched, 2)
        print(f"image {i}: bpp {float(res['bpp']):.4f}  {time.time() - t0:.1f}s  "
              f"|c| {np.abs(res['vae_c']).max():.2f} |y| {np.abs(res['y']).max():.2f} "
              f"|eps| {np.abs(res['eps']).max():.2f} |x_dec| {np.abs(res['x_dec']).max():.2f} "
              f"syms {res['symbols'].size} range [{res['symbols'].min()}, {res['symbols'].max()}] "
              f"idx range [{res['indexes'].min()}, {res['indexes'].max()}]")
        fixtures[f"img{i}_in"] = img
        for k, v in res.items():
            fixtures[f"img{i}_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "e2e_128.npz"), **fixtures)
    print("wrote", os.path.join(HERE, "e2e_128.npz"))


if __name__ == "__main__":
    main()
