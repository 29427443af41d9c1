"""Command-line codec with the reference's interface (reference inference.py:94-147).

    python inference.py --input DIR --output DIR [--ckpt FILE] [--steps 2] [--seed 231]

Per image: pad to x64 -> compress to `<output>/data/<stem>` (reference file format) ->
decompress -> q_sample at t=used_timesteps-1 -> relay DDIM -> VAE decode -> crop -> PNG.
Differences from the reference, all forced by the offline image:
  * no checkpoint is shipped: without --ckpt the model uses the seeded synthetic weights;
    with --ckpt, a plain state dict is read with torch.load(weights_only=True);
  * the OpenCLIP "" embedding (reference :122) is replaced by the seeded synthetic context;
  * the noise draws (x_T, q_sample noise, and the spaced sampler's per-step randn_like) come from a
    seeded CPU generator in the reference's order, not from the device RNG.
The noise draws follow the reference order (inference.py:64-65: a discarded randn, then noise).
"""
import os
import sys
from argparse import ArgumentParser, Namespace
from typing import List, Tuple

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

IMG_EXTS = (".jpg", ".png", ".jpeg")


def pad(img: np.ndarray, scale: int) -> np.ndarray:
    """Zero-pad bottom/right to a multiple of `scale` (reference utils/image/common.py:251-258)."""
    h, w = img.shape[:2]
    ph, pw = (-h) % scale, (-w) % scale
    return np.pad(img, ((0, ph), (0, pw), (0, 0)), mode="constant", constant_values=0)


def list_image_files(img_dir: str, follow_links: bool = True) -> List[str]:
    files = []
    for dir_path, _, names in os.walk(img_dir, followlinks=follow_links):
        files += [os.path.join(dir_path, n) for n in names if os.path.splitext(n)[1].lower() in IMG_EXTS]
    return files


@torch.no_grad()
def process(model, imgs: List[np.ndarray], sampler: str, steps: int, stream_path: str, guidance_scale: float,
            c_crossattn: List[torch.Tensor], generator: torch.Generator) -> Tuple[List[np.ndarray], float]:
    """reference inference.py:22-91 on the HIP path."""
    from rdeic_amd.ddim_sampler_relay import DDIMSampler
    from rdeic_amd.spaced_sampler_relay import SpacedSampler
    n = len(imgs)
    control = torch.tensor(np.stack(imgs) / 255.0, dtype=torch.float32).clamp_(0, 1)
    control = control.permute(0, 3, 1, 2).contiguous().to(model.device)
    H, W = control.shape[-2:]
    bpp = model.apply_condition_compress(control, stream_path, H, W)
    c_latent, guide_hint = model.apply_condition_decompress(stream_path)
    cond = {"c_latent": [c_latent], "c_crossattn": c_crossattn, "guide_hint": guide_hint}
    shape = (n, 4, H // 8, W // 8)
    torch.randn(shape, generator=generator)  # the reference's discarded x_T draw
    noise = torch.randn(shape, generator=generator).to(model.device)
    t = torch.full((n,), model.used_timesteps - 1, dtype=torch.long, device=model.device)
    x_T = model.q_sample(x_start=c_latent, t=t, noise=noise)
    if sampler == "ddpm":
        step_noise = [torch.randn(shape, generator=generator) for _ in range(steps)]
        samples = SpacedSampler(model, var_type="fixed_small").sample(
            steps, shape, cond, unconditional_guidance_scale=guidance_scale, unconditional_conditioning=None,
            cond_fn=None, x_T=x_T, step_noise=step_noise)
    else:
        samples, _ = DDIMSampler(model).sample(S=steps, batch_size=n, shape=shape[1:], conditioning=cond,
                                               unconditional_conditioning=None,
                                               unconditional_guidance_scale=guidance_scale, x_T=x_T, eta=0)
    x = model.decode_first_stage(samples)
    x = ((x + 1) / 2).clamp(0, 1)
    x = (x.permute(0, 2, 3, 1) * 255).cpu().numpy().clip(0, 255).astype(np.uint8)
    return [x[i] for i in range(n)], bpp


def parse_args(argv=None) -> Namespace:
    p = ArgumentParser()
    p.add_argument("--ckpt", default="", type=str, help="state dict (.pt/.ckpt, tensors only); empty = synthetic")
    p.add_argument("--config", default="", type=str, help="accepted for compatibility (architecture is fixed)")
    p.add_argument("--input", type=str, required=True)
    p.add_argument("--sampler", type=str, default="ddpm", choices=["ddpm", "ddim"])
    p.add_argument("--steps", default=2, type=int)
    p.add_argument("--guidance_scale", default=1.0, type=float)
    p.add_argument("--output", type=str, default="results/")
    p.add_argument("--seed", type=int, default=231)
    p.add_argument("--device", type=str, default="cuda", choices=["cuda"])
    p.add_argument("--dtype", type=str, default="fp32", choices=["fp32", "bf16"])
    return p.parse_args(argv)


def load_model(ckpt: str, dtype: str):
    from rdeic_amd.rdeic import RDEIC
    model = RDEIC(compute_dtype=torch.float32 if dtype == "fp32" else torch.bfloat16)
    if ckpt:
        sd = torch.load(ckpt, map_location="cpu", weights_only=True)
        sd = sd.get("state_dict", sd)
        model.load_state_dict(sd, strict=True)
    else:
        model.init_synthetic()
    model.preprocess_model.update(force=True)
    return model


def main(argv=None) -> None:
    from PIL import Image
    from rdeic_amd.synthetic import synth_context
    args = parse_args(argv)
    if not os.path.isdir(args.input):
        raise SystemExit(f"--input {args.input} is not a directory")
    gen = torch.Generator().manual_seed(args.seed)
    model = load_model(args.ckpt, args.dtype)
    c_crossattn = [synth_context().to(model.device)]
    print(f"sampling {args.steps} steps using {args.sampler} sampler")
    bpps = []
    for file_path in list_image_files(args.input):
        img = Image.open(file_path).convert("RGB")
        x = pad(np.array(img), scale=64)
        save_path = os.path.join(args.output, os.path.relpath(file_path, args.input))
        parent, name = os.path.split(save_path)
        stem = os.path.splitext(name)[0]
        os.makedirs(os.path.join(parent, "data"), exist_ok=True)
        preds, bpp = process(model, [x], args.sampler, args.steps, os.path.join(parent, "data", stem),
                             args.guidance_scale, c_crossattn, gen)
        out_path = os.path.join(parent, f"{stem}.png")
        Image.fromarray(preds[0][:img.height, :img.width, :]).save(out_path)
        bpps.append(bpp)
        print(f"save to {out_path}, bpp {bpp}")
    if bpps:
        print(f"avg bpp: {sum(bpps) / len(bpps)}")


if __name__ == "__main__":
    main()
