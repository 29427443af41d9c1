"""Golden vectors of ONE adapter fine-tune step (config 5, §8f rank 1), produced by the REFERENCE's
own modules and torch autograd on CPU, fp32, at 128x128 (16x16 latent), batch 1.

Run in the development container only (the reference does not exist on the GPU box):
    python -m tests.golden.make_train_golden [SIZE]
Output (committed): tests/golden/train_128.npz, and train_512.npz at config 5's own size (r04).

The step restates LatentDiffusion.get_input (ddpm.py:777-833: encode_hc under no_grad, the
posterior sample x 0.18215, h = c x 0.18215) + RDEIC.get_input (model/rdeic.py:678-686: the
Compression forward in training mode, bpp / q_bpp from the likelihoods) + RDEIC.forward /
p_losses non-refine branch (rdeic.py:774-835, eps parameterization, logvar 0) with
configs/model/rdeic_finetune_ood.yaml's weights (l_guide_weight 3, l_bpp_weight 1, lr 2e-5,
sd_locked: the base UNet frozen), then configure_optimizers' AdamW (rdeic.py:763-772) for one step.
The UNet, NoiseEstimator, Compression (incl. VectorQuantiser.forward with its contrastive loss
and dead-code re-init, compression_modules.py:228-307), VAE encoder run as the reference's code;
compressai's GaussianConditional training forward / LowerBound are restated in
oracle/train_ref.py (compressai is absent).

Stored: the draws, every loss term, c_latent / x_start / x_noisy / model eps, the VQ state after
the forward (embedding checksum, embed_prob, indices), and per trainable tensor of the control
model and the compressor: the gradient's sum, L2 norm and 4 seeded random projections
(proj_seed(name)), full gradients of a few small tensors, and the AdamW-updated values of those.
"""
from __future__ import annotations

import math
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import train_ref  # noqa: E402
from rdeic_amd.config import CONFIG  # noqa: E402
from rdeic_amd.synthetic import synth_context, synth_image, train_draws  # noqa: E402
from tests.golden import refload  # noqa: E402
from tests.golden.make_golden import fill_module, schedule  # noqa: E402
from tests.golden.train_proj import projections  # noqa: E402

SIZE = int(sys.argv[1]) if len(sys.argv) > 1 else 128
# "f64" as the second argument: the same step in float64 (r05, the conditioning of the fp32 gradients):
# writes train_{SIZE}_f64.npz with the loss terms and every gradient's sum / norm / projections only
F64 = len(sys.argv) > 2 and sys.argv[2] == "f64"
DT = torch.float64 if F64 else torch.float32
SEED = 5
L_GUIDE, L_BPP, LR = 3.0, 1.0, 2e-5
FULL_GRADS = ("control_model.control_model.input_blocks.0.0.weight", "control_model.enc_zero_convs_out.0.0.weight",
              "control_model.middle_block_out.0.bias", "control_model.control_model.time_embed.0.bias",
              "control_model.control_model.input_blocks.1.1.transformer_blocks.0.norm1.weight",
              "control_model.control_model.input_blocks.1.0.in_layers.0.weight",
              "preprocess_model.out.weight", "preprocess_model.out.bias",
              "preprocess_model.entropy_parameters_anchor.0.fusion.4.weight",
              "preprocess_model.local_context.3.weight", "preprocess_model.hyper_dec.hyper_dec.0.subpel_conv.0.bias",
              "preprocess_model.decoder.g_s.0.bias")


def main():
    torch.set_num_threads(os.cpu_count() or 8)
    R = refload.load()
    cfg = CONFIG
    unet = R.UNetModel(**cfg["unet"])
    ne = R.NoiseEstimator(**cfg["control"])
    enc = R.Encoder(**cfg["ddconfig"]).eval()
    quant_conv = torch.nn.Conv2d(8, 8, 1)
    comp = R.Compression(**cfg["compression"])
    for m, p in [(unet, "model.diffusion_model."), (ne, "control_model."), (enc, "first_stage_model.encoder."),
                 (quant_conv, "first_stage_model.quant_conv."), (comp, "preprocess_model.")]:
        fill_module(m, p)
    for m in (unet, ne, enc, quant_conv, comp):
        m.to(DT)
    if F64:  # the reference casts to the UNets' `dtype` attribute and builds the timestep embedding in fp32
        for m in (unet, ne):
            for sub in m.modules():
                if isinstance(getattr(sub, "dtype", None), torch.dtype) and "dtype" in vars(sub):
                    sub.dtype = DT
        for mod in list(sys.modules.values()):
            f = getattr(mod, "timestep_embedding", None) if mod is not None else None
            if callable(f) and not getattr(f, "_f64", False):
                def emb64(*a, _f=f, **k):
                    return _f(*a, **k).to(DT)
                emb64._f64 = True
                setattr(mod, "timestep_embedding", emb64)
        import types
        for mod in list(sys.modules.values()):  # the CrossAttention fp32 upcast of q, k: skipped in f64
            if mod is not None and getattr(mod, "_ATTN_PRECISION", None) == "fp32":
                mod._ATTN_PRECISION = "f64"
        for m in (unet, ne, comp):  # GroupNorm32.forward upcasts to fp32 (x.float()): the plain GroupNorm instead
            for sub in m.modules():
                if isinstance(sub, torch.nn.GroupNorm) and type(sub) is not torch.nn.GroupNorm:
                    sub.forward = types.MethodType(torch.nn.GroupNorm.forward, sub)
        for obj in (ne,):  # NoiseEstimator's globals (AST-extracted module dict)
            g = type(obj).forward.__globals__
            f = g.get("timestep_embedding")
            if callable(f) and not getattr(f, "_f64", False):
                g["timestep_embedding"] = lambda *a, _f=f, **k: _f(*a, **k).to(DT)
    for m in (unet, enc, quant_conv):
        m.requires_grad_(False)
    unet.train(), ne.train(), comp.train()
    sched = schedule(R)
    ac = sched["alphas_cumprod"].double().numpy()
    sched = {k: v.to(DT) for k, v in sched.items()}
    f32 = lambda a: torch.tensor(a, dtype=DT)  # noqa: E731
    sqrt_recip = f32(np.sqrt(1.0 / ac))
    sqrt_recipm1 = f32(np.sqrt(1.0 / ac - 1))
    lamba = sqrt_recipm1[cfg["used_timesteps"] - 1]

    img = synth_image(SIZE, SIZE, 231)
    ctx = synth_context().to(DT)
    hl = SIZE // 8
    dr = train_draws(1, hl, hl, cfg["compression"]["slice_ch"], SEED, cfg["used_timesteps"])
    dr = {k: ([s.to(DT) for s in v] if isinstance(v, list) else (v.to(DT) if v.is_floating_point() else v))
          for k, v in dr.items()}
    t = dr["t"]
    out = {"image": img, "t": t.numpy(), "post_eps": dr["post_eps"].numpy(),
           "noise": dr["noise"].numpy()}
    for i, s in enumerate(dr["slice_noise"]):
        out[f"slice_noise{i}"] = s.numpy()
    t0 = time.time()
    x = torch.tensor(img[None] / 255.0, dtype=DT).permute(0, 3, 1, 2).contiguous()
    with torch.no_grad():  # LatentDiffusion.get_input / encode_first_stage (ddpm.py:777-789, 857-860)
        h_out, c = enc.forward_hc(x * 2 - 1)
        moments = quant_conv(h_out)
        mean, logvar = torch.chunk(moments, 2, dim=1)
        logvar = torch.clamp(logvar, -30.0, 20.0)
        std = torch.exp(0.5 * logvar)
        x_start = cfg["scale_factor"] * (mean + std * dr["post_eps"])
        h = cfg["scale_factor"] * c
    if F64:  # tensors the reference creates inside its forward (VQ one-hot encodings) follow the default dtype
        torch.set_default_dtype(torch.float64)
    train_ref.NOISE_QUEUE[:] = list(dr["slice_noise"])
    c_latent, lik, qlik, emb_loss, guide_hint = comp(h)
    assert not train_ref.NOISE_QUEUE
    N, _, H, W_ = x_start.shape
    num_pixels = N * H * W_ * 64
    bpp = sum((torch.log(l_).sum() / (-math.log(2) * num_pixels)) for l_ in lik)
    q_bpp = sum((torch.log(l_).sum() / (-math.log(2) * num_pixels)) for l_ in qlik)
    noise = dr["noise"] + (c_latent - x_start) / lamba
    x_noisy = (sched["sqrt_alphas_cumprod"][t].view(-1, 1, 1, 1) * x_start +
               sched["sqrt_one_minus_alphas_cumprod"][t].view(-1, 1, 1, 1) * noise)
    eps = ne(x=x_noisy, timesteps=t, context=ctx, guide_hint=guide_hint, base_model=unet)
    model_output = sqrt_recip[t].view(-1, 1, 1, 1) * x_noisy - sqrt_recipm1[t].view(-1, 1, 1, 1) * eps
    loss_simple = torch.nn.functional.mse_loss(x_start, model_output, reduction="none").mean([1, 2, 3])
    loss = L_GUIDE * loss_simple.mean()
    loss = loss + L_BPP * bpp
    loss = loss + L_BPP * emb_loss
    loss_guide = torch.nn.functional.mse_loss(x_start, c_latent)
    loss = loss + L_GUIDE * loss_guide
    print(f"forward {time.time() - t0:.1f}s loss {loss.item():.6f} simple {loss_simple.mean().item():.6f} "
          f"bpp {bpp.item():.4f} q_bpp {q_bpp.item():.4f} emb {emb_loss.item():.6f} guide {loss_guide.item():.6f}")
    E_after_fwd = comp.quantize.embedding.weight.detach().clone()
    t0 = time.time()
    loss.backward()
    print(f"backward {time.time() - t0:.1f}s")
    for k, v in dict(loss=loss, l_simple=loss_simple.mean(), l_bpp=bpp, q_bpp=q_bpp, l_emb=emb_loss,
                     l_guide=loss_guide).items():
        out["loss_" + k] = np.float64(v.item())
    # above 128^2 the spatial intermediates are stored on a stride-SUB pixel grid (the whole 512^2 set
    # would be 16 MB); the GPU test subsamples its own tensors the same way
    sub = 1 if SIZE <= 128 else 4
    sp = lambda t: np.ascontiguousarray(t.detach().numpy()[:, :, ::sub, ::sub])  # noqa: E731
    out.update(x_start=sp(x_start), h=sp(h), c_latent=sp(c_latent), guide_hint=sp(guide_hint), x_noisy=sp(x_noisy),
               eps=sp(eps), y_lik=sp(lik[0]), lamba=np.float32(lamba.item()), subsample=np.int64(sub))
    q = comp.quantize
    out["vq_embed_prob"] = q.embed_prob.numpy().copy()
    out["vq_E_after_fwd_rowsum"] = E_after_fwd.double().sum(1).numpy()
    out["vq_E_after_fwd_sq"] = np.float64((E_after_fwd.double() ** 2).sum().item())
    names, sums, norms, projs = [], [], [], []
    params = []
    for mod, prefix in ((ne, "control_model."), (comp, "preprocess_model.")):
        for k, p in mod.named_parameters():
            full = prefix + k
            g = p.grad if p.grad is not None else torch.zeros_like(p)
            names.append(full)
            sums.append(g.double().sum().item())
            norms.append(g.double().norm().item())
            projs.append(projections(full, g))
            params.append((full, p))
            if full in FULL_GRADS:
                out["grad:" + full] = g.numpy().copy()
    out["grad_names"] = np.asarray(names)
    out["grad_sum"] = np.asarray(sums)
    out["grad_norm"] = np.asarray(norms)
    out["grad_proj"] = np.stack(projs)
    if F64:
        path = os.path.join(HERE, f"train_{SIZE}_f64.npz")
        np.savez_compressed(path, **{k: v for k, v in out.items() if k.startswith("loss_") or k.startswith("grad_")})
        print("wrote", path)
        return
    # AdamW step (torch.optim.AdamW defaults, lr from the fine-tune config)
    opt = torch.optim.AdamW([p for _, p in params], lr=LR)
    opt.step()
    for full, p in params:
        if full in FULL_GRADS:
            out["after_adamw:" + full] = p.detach().numpy().copy()
    out["after_adamw_E_rowsum"] = comp.quantize.embedding.weight.detach().double().sum(1).numpy()
    # the reference's own AdamW and the restated one agree (the restatement is what the GPU test mirrors)
    path = os.path.join(HERE, f"train_{SIZE}.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, f"{os.path.getsize(path) / 1e6:.2f} MB; {len(names)} trainable tensors, "
          f"{sum(p.numel() for _, p in params) / 1e6:.2f}M params")


if __name__ == "__main__":
    main()
