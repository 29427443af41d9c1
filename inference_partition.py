"""Batched command-line codec with the reference's inference_partition.py interface
(reference inference_partition.py:139-318 process(), :320-352 arguments, :355-571 main()).

    python inference_partition.py --input DIR --output DIR [--batch_size 8] [--micro_batch_size 4]
        [--steps 2] [--sampler ddpm|ddim] [--bf16 | --fp16] [--enable_resize_guard --max_long_side 1024
        --upsample_to_original] [--save_intermediates] [--max_images N]

What it keeps from the reference:
  * images are grouped by their padded (multiple-of-64) working size after the optional resize
    guard (LANCZOS downscale so max(H, W) <= --max_long_side), sorted, and processed in batches of
    --batch_size within a group (:389-458);
  * every image is compressed to its own bitstream file `<output>/<rel>/data/<stem>` and decoded
    back from that file (:173-180), bpp = 8 * filesize / (padded H * W);
  * relay sampling + VAE decoding run over micro-batches of --micro_batch_size (:244-317), with
    classifier-free guidance when an unconditional context is given;
  * outputs are cropped to the working size, optionally upsampled back to the original size with
    --upsample_method, saved as PNG, and scored: `<output>/metrics.csv` with the reference's columns
    image, bpp, scale, psnr, ssim, ms_ssim, lpips (:540-571);
  * --save_intermediates writes the decoded latent (.pt / .npy), a guide-hint preview and a
    preview decode of c_latent per image (:188-233); --profile_memory prints device memory.
What differs, all forced by the offline image or by design:
  * captioning (--use_captions, Qwen2-VL) and OpenCLIP text encoding are out of scope: the seeded
    synthetic context stands in for the "" embedding, and --use_captions is refused;
  * --bf16 selects the bf16 compute path; the default is the fp32 parity path. The reference's
    --fp16 (autocast float16) is accepted and selects the same bf16 path with a notice on stderr:
    no float16 kernels are built for MI355X;
  * LPIPS needs an AlexNet backbone that is not available offline: the column is NaN; PSNR, SSIM
    and MS-SSIM are computed on the device (rdeic_amd/metrics.py);
  * noise comes from a CPU generator seeded per image (--seed + the image's index in sorted
    order), so results do not depend on how images are grouped into batches and micro-batches.
"""
import csv
import os
import sys
import time
from argparse import ArgumentParser, Namespace
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from inference import list_image_files, load_model, pad  # noqa: E402

RESAMPLE = {"lanczos": "LANCZOS", "bicubic": "BICUBIC", "bilinear": "BILINEAR", "nearest": "NEAREST"}


def image_noise(shape, seed: int, steps: int, sampler: str):
    """(noise, per-step noise or None) for one image, in the reference's draw order: a discarded
    x_T randn, the q_sample noise, then one randn per spaced-sampler step."""
    g = torch.Generator().manual_seed(int(seed))
    torch.randn(shape, generator=g)
    noise = torch.randn(shape, generator=g)
    steps_noise = [torch.randn(shape, generator=g) for _ in range(steps)] if sampler == "ddpm" else None
    return noise, steps_noise


@torch.no_grad()
def process(model, imgs: List[np.ndarray], sampler: str, steps: int, stream_paths: List[str], guidance_scale: float,
            c_crossattn: List[torch.Tensor], uc_crossattn: Optional[List[torch.Tensor]] = None,
            micro_batch_size: Optional[int] = None, seeds: Optional[List[int]] = None, profile_memory: bool = False,
            save_intermediates: bool = False, intermediate_prefixes: Optional[List[str]] = None,
            latent_format: str = "pt") -> Tuple[List[np.ndarray], List[float]]:
    """reference inference_partition.py:139-318 on the HIP path: per-image compress -> file ->
    decompress, then relay sampling + VAE decode in micro-batches."""
    from rdeic_amd.ddim_sampler_relay import DDIMSampler
    from rdeic_amd.spaced_sampler_relay import SpacedSampler
    n = len(imgs)
    if n != len(stream_paths):
        raise ValueError("imgs and stream_paths must have the same length")
    seeds = list(seeds) if seeds is not None else list(range(n))
    control = torch.tensor(np.stack(imgs) / 255.0, dtype=torch.float32).clamp_(0, 1).permute(0, 3, 1, 2).contiguous()
    H, W = control.shape[-2:]
    bpps, c_lats, hints = [], [], []
    _mem(profile_memory, "before compress")
    for i in range(n):
        bpps.append(model.apply_condition_compress(control[i:i + 1].to(model.device), stream_paths[i], H, W))
        c_lat, hint = model.apply_condition_decompress(stream_paths[i])
        c_lats.append(c_lat)
        hints.append(hint)
        if save_intermediates:
            _save_intermediates(model, intermediate_prefixes[i], c_lat, hint, latent_format)
    c_latent, guide_hint = torch.cat(c_lats), torch.cat(hints)
    chunk = micro_batch_size or n
    preds: List[np.ndarray] = []
    _mem(profile_memory, "before sampling")
    for s0 in range(0, n, chunk):
        s1 = min(s0 + chunk, n)
        bs = s1 - s0
        shape = (bs, 4, H // 8, W // 8)
        draws = [image_noise((1,) + shape[1:], seeds[j], steps, sampler) for j in range(s0, s1)]
        noise = torch.cat([d[0] for d in draws]).to(model.device)
        ctx = _slice_ctx(c_crossattn, s0, s1)
        cond = {"c_latent": [c_latent[s0:s1]], "c_crossattn": ctx, "guide_hint": guide_hint[s0:s1]}
        uc = None
        if uc_crossattn is not None:
            uc = {"c_latent": [c_latent[s0:s1]], "c_crossattn": _slice_ctx(uc_crossattn, s0, s1),
                  "guide_hint": guide_hint[s0:s1]}
        t = torch.full((bs,), model.used_timesteps - 1, dtype=torch.long, device=model.device)
        x_T = model.q_sample(x_start=c_latent[s0:s1], t=t, noise=noise)
        if sampler == "ddpm":
            step_noise = [torch.cat([d[1][k] for d in draws]) for k in range(steps)]
            samples = SpacedSampler(model, var_type="fixed_small").sample(
                steps, shape, cond, unconditional_guidance_scale=guidance_scale, unconditional_conditioning=uc,
                cond_fn=None, x_T=x_T, step_noise=step_noise)
        else:
            samples, _ = DDIMSampler(model).sample(S=steps, batch_size=bs, shape=shape[1:], conditioning=cond,
                                                   unconditional_conditioning=uc,
                                                   unconditional_guidance_scale=guidance_scale, x_T=x_T, eta=0)
        x = model.decode_first_stage(samples)
        x = ((x + 1) / 2).clamp(0, 1)
        x = (x.permute(0, 2, 3, 1) * 255).cpu().numpy().clip(0, 255).astype(np.uint8)  # truncating cast (:85-87)
        preds.extend(x[i] for i in range(bs))
        _mem(profile_memory, f"after chunk {s0}-{s1}")
    return preds, bpps


def _slice_ctx(ctx: List[torch.Tensor], s0: int, s1: int) -> List[torch.Tensor]:
    if ctx and hasattr(ctx[0], "shape") and ctx[0].shape[0] > 1:
        return [ctx[0][s0:s1]]
    return ctx


def _mem(on: bool, what: str) -> None:
    if on and torch.cuda.is_available():
        print(f"[mem] {what}: alloc={torch.cuda.memory_allocated() / 1e9:.3f} GB, "
              f"reserved={torch.cuda.memory_reserved() / 1e9:.3f} GB")


def _save_intermediates(model, prefix: str, c_lat: torch.Tensor, hint: torch.Tensor, latent_format: str) -> None:
    from PIL import Image
    lat = c_lat.detach().cpu()
    if latent_format == "npy":
        np.save(f"{prefix}_latent.npy", lat.numpy())
    else:
        torch.save(lat, f"{prefix}_latent.pt")
    gh = hint.detach().float().cpu()[0]
    gh = (gh - gh.min()) / (gh.max() - gh.min() + 1e-8)
    vis = gh[:3] if gh.shape[0] >= 3 else gh[:1].repeat(3, 1, 1)
    Image.fromarray((vis.permute(1, 2, 0).numpy() * 255.0).clip(0, 255).astype(np.uint8)).save(f"{prefix}_guide.png")
    dec = ((model.decode_first_stage(c_lat) + 1) / 2).clamp(0, 1)
    dec = (dec.permute(0, 2, 3, 1).cpu().numpy() * 255.0).clip(0, 255).astype(np.uint8)
    Image.fromarray(dec[0]).save(f"{prefix}_compressed.png")


def compute_metrics(pred: np.ndarray, target: np.ndarray) -> Dict[str, float]:
    """reference inference_partition.py:28-70 (pyiqa psnr / ssim / ms_ssim / lpips), on the device."""
    from rdeic_amd import metrics
    p = torch.from_numpy(np.ascontiguousarray(pred[None])).cuda()
    t = torch.from_numpy(np.ascontiguousarray(target[None])).cuda()
    out = {"psnr": float(metrics.psnr(p, t)[0]), "ssim": float("nan"), "ms_ssim": float("nan"),
           "lpips": float("nan")}
    if min(pred.shape[:2]) >= 176:
        s, ms = metrics.ssim_ms_ssim(p, t)
        out.update(ssim=float(s[0]), ms_ssim=float(ms[0]))
    elif min(pred.shape[:2]) >= 11:
        out.update(ssim=float(metrics.ssim_levels(p, t, 1)[0, 0, 0]))
    return out


def parse_args(argv=None) -> Namespace:
    p = ArgumentParser()
    p.add_argument("--ckpt_sd", default="", type=str, help="SD state dict (tensors only); empty = synthetic")
    p.add_argument("--ckpt_cc", default="", type=str, help="compression + control state dict; merged over --ckpt_sd")
    p.add_argument("--config", default="", type=str, help="accepted for compatibility (architecture is fixed)")
    p.add_argument("--input", type=str, required=True)
    p.add_argument("--sampler", type=str, default="ddpm", choices=["ddpm", "ddim"])
    p.add_argument("--steps", default=2, type=int)
    p.add_argument("--guidance_scale", default=1.0, type=float)
    p.add_argument("--output", type=str, default="results/")
    p.add_argument("--seed", type=int, default=231)
    p.add_argument("--device", type=str, default="cuda", choices=["cuda"])
    p.add_argument("--max_images", type=int, default=0, help="if > 0, process only the first N images in sorted order")
    p.add_argument("--use_captions", action="store_true", help="(refused: Qwen2-VL captioning needs weights)")
    p.add_argument("--batch_size", type=int, default=1, help="images processed together (grouped by resolution)")
    p.add_argument("--micro_batch_size", type=int, default=0, help="chunks of the sampling / decoding stage")
    p.add_argument("--bf16", action="store_true", help="bf16 compute path (default: fp32 parity path)")
    p.add_argument("--fp16", action="store_true",
                   help="the reference's reduced-precision switch (autocast float16); here it selects the bf16 "
                        "path, with a notice: no float16 kernels are built for MI355X")
    p.add_argument("--profile_memory", action="store_true")
    p.add_argument("--save_intermediates", action="store_true")
    p.add_argument("--latent_format", type=str, default="pt", choices=["pt", "npy"])
    p.add_argument("--max_long_side", type=int, default=0)
    p.add_argument("--enable_resize_guard", action="store_true")
    p.add_argument("--upsample_to_original", action="store_true")
    p.add_argument("--upsample_method", type=str, default="lanczos", choices=list(RESAMPLE))
    p.add_argument("--suppress_warnings", action="store_true")
    args = p.parse_args(argv)
    if args.fp16:
        print("[inference_partition] --fp16: the reduced-precision path computes in bf16 on MI355X "
              "(float16 autocast is not provided); same as --bf16", file=sys.stderr)
        args.bf16 = True
    return args


def _load(args):
    if args.ckpt_sd or args.ckpt_cc:
        sd = {}
        for path in (args.ckpt_sd, args.ckpt_cc):
            if path:
                part = torch.load(path, map_location="cpu", weights_only=True)
                sd.update(part.get("state_dict", part))
        from rdeic_amd.rdeic import RDEIC
        model = RDEIC(compute_dtype=torch.bfloat16 if args.bf16 else torch.float32)
        model.load_state_dict(sd, strict=False)
        model.preprocess_model.update(force=True)
        return model
    return load_model("", "bf16" if args.bf16 else "fp32")


def main(argv=None) -> List[Dict]:
    from PIL import Image
    from rdeic_amd.synthetic import synth_context
    args = parse_args(argv)
    if args.use_captions:
        raise SystemExit("--use_captions needs the Qwen2-VL captioner and OpenCLIP weights, not available offline")
    if not os.path.isdir(args.input):
        raise SystemExit(f"--input {args.input} is not a directory")
    if args.suppress_warnings:
        import warnings
        warnings.filterwarnings("ignore")
    model = _load(args)
    ctx = synth_context().to(model.device)
    os.makedirs(args.output, exist_ok=True)
    print(f"sampling {args.steps} steps using {args.sampler} sampler")
    files = sorted(list_image_files(args.input))
    if args.max_images > 0:
        files = files[:args.max_images]
    order = {f: k for k, f in enumerate(files)}
    groups: Dict[Tuple[int, int], List[str]] = {}
    meta: Dict[str, dict] = {}
    for f in files:
        with Image.open(f) as im:
            w, h = im.size
        scale, sw, sh = 1.0, w, h
        if args.enable_resize_guard and args.max_long_side > 0 and max(w, h) > args.max_long_side:
            scale = args.max_long_side / max(w, h)
            sw, sh = max(1, int(round(w * scale))), max(1, int(round(h * scale)))
        key = (((sh + 63) // 64) * 64, ((sw + 63) // 64) * 64)
        groups.setdefault(key, []).append(f)
        meta[f] = {"orig_h": h, "orig_w": w, "scaled_h": sh, "scaled_w": sw, "scale": scale}
    records, bpps = [], []
    resample = getattr(Image, RESAMPLE[args.upsample_method])
    for key in sorted(groups):
        paths = sorted(groups[key])
        for b0 in range(0, len(paths), max(1, args.batch_size)):
            batch = paths[b0:b0 + max(1, args.batch_size)]
            imgs, streams, prefixes, targets = [], [], [], []
            for f in batch:
                full = Image.open(f).convert("RGB")
                m = meta[f]
                scaled = full if full.size == (m["scaled_w"], m["scaled_h"]) else \
                    full.resize((m["scaled_w"], m["scaled_h"]), Image.LANCZOS)
                imgs.append(pad(np.array(scaled), scale=64))
                rel = os.path.relpath(f, args.input)
                parent = os.path.dirname(os.path.join(args.output, rel))
                stem = os.path.splitext(os.path.basename(rel))[0]
                os.makedirs(os.path.join(parent, "data"), exist_ok=True)
                streams.append(os.path.join(parent, "data", stem))
                prefixes.append(os.path.join(parent, stem))
                targets.append((np.array(full), np.array(scaled), rel))
            t0 = time.time()
            preds, bpp_batch = process(model, imgs, args.sampler, args.steps, streams, args.guidance_scale, [ctx],
                                       micro_batch_size=args.micro_batch_size or None,
                                       seeds=[args.seed + order[f] for f in batch],
                                       profile_memory=args.profile_memory, save_intermediates=args.save_intermediates,
                                       intermediate_prefixes=prefixes, latent_format=args.latent_format)
            per_image = (time.time() - t0) / len(batch)
            for f, pred, (orig, scaled, rel), prefix, bpp in zip(batch, preds, targets, prefixes, bpp_batch):
                m = meta[f]
                out = Image.fromarray(pred[:m["scaled_h"], :m["scaled_w"], :])
                up = args.enable_resize_guard and args.upsample_to_original and m["scale"] < 1.0
                if up:
                    out = out.resize((m["orig_w"], m["orig_h"]), resample)
                out.save(f"{prefix}.png")
                vals = compute_metrics(np.array(out), orig if up else scaled)
                records.append({"image": rel, "bpp": bpp, "scale": m["scale"], **vals})
                bpps.append(bpp)
                print(f"save to {prefix}.png, bpp {bpp:.3f}, PSNR {vals['psnr']:.2f}dB, SSIM {vals['ssim']:.4f}, "
                      f"LPIPS {vals['lpips']:.4f}, time {per_image:.2f}s")
    if bpps:
        print(f"avg bpp: {sum(bpps) / len(bpps)}")
    if records:
        path = os.path.join(args.output, "metrics.csv")
        with open(path, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=["image", "bpp", "scale", "psnr", "ssim", "ms_ssim", "lpips"])
            w.writeheader()
            w.writerows(records)
        for k in ("psnr", "ssim", "ms_ssim", "lpips"):
            v = np.array([r[k] for r in records], dtype=np.float64)
            print(f"Mean {k.upper()}: {np.nanmean(v) if np.isfinite(v).any() else float('nan'):.4f}")
        print(f"Metrics saved to {path}")
    return records


if __name__ == "__main__":
    main()
