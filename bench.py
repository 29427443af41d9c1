"""Benchmark: 512x512 images/s through the full RDEIC hot path on N MI355X GPUs.

One step = one batch of B synthetic 512x512 images per GPU through
  encode (VAE) -> entropy model + rANS/torchac to bytes -> bytes back through the entropy
  decoder -> relay DDIM (S steps, UNet + control) -> VAE decode -> uint8
plus the per-image metric rows (bpp, bytes, PSNR) and ONE all-gather of them across ranks.
Data: synthetic (seeded smooth images, random-init weights of the real architecture, a seeded
[1, 77, 1024] text context) — no datasets or checkpoints offline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 16] [--size 512] [--ddim-steps 2]
For N > 1 launch with torch.distributed.run (one process per GPU, RCCL).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP32_TFLOPS = 157.3
PEAK_HBM_GBS = 8000.0


def conv_traffic():
    """HBM bytes per conv launch, from the latest committed PMC run (tools/pmc_bench.sh ->
    profiles/conv_traffic.json: FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction of
    MI355X_MICROARCH.md §HBM). Counters cannot be read inside this process, so the figure is the
    measured one with its source, or None when no PMC run has been committed."""
    try:
        with open(os.path.join(ROOT, "profiles", "conv_traffic.json")) as f:
            t = json.load(f)
        return {"bytes_per_launch": t["bytes_per_launch"], "algorithmic_flops_per_launch": t.get("flops_per_launch"),
                "source": t.get("source", "profiles/conv_traffic.json")}
    except (OSError, ValueError, KeyError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=16, help="images per GPU per step")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--ddim-steps", type=int, default=2, help="relay sampler steps")
    ap.add_argument("--sampler", default="ddim", choices=["ddim", "ddpm"],
                    help="relay sampler (config 2 names 2-step relay DDIM; ddpm = the CLI's spaced sampler)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--prof-every", type=int, default=8,
                    help="roofline timing: every launch >= 50 GFLOP (64 MB for GroupNorm), and a hashed "
                         "1-in-N sample of the smaller ones (weighted estimate)")
    ap.add_argument("--coder-groups", type=int, default=None,
                    help="image groups interleaved in the entropy-stage loops (default: the library's)")
    ap.add_argument("--no-plans", action="store_true", help="eager launches (no launch-plan replay), A/B only")
    ap.add_argument("--no-geglu-fuse", action="store_true", help="unfused GEGLU (projection + geglu kernel), A/B only")
    ap.add_argument("--rate-gain", type=float, default=None,
                    help="synthetic bpp knob (rdeic_amd/weights.py); default: the ~0.08 bpp gain of config 2")
    return ap.parse_args()


def main():
    args = parse()
    from rdeic_amd import ops, parallel
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image

    rank, world, local = parallel.init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B, S = args.batch, args.size
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    from rdeic_amd import weights as W
    rate_gain = W.RATE_GAIN_BPP008 if args.rate_gain is None else args.rate_gain
    model = RDEIC(compute_dtype=dtype, device=dev).init_synthetic(rate_gain=rate_gain)
    model.preprocess_model.update(force=True)
    if args.coder_groups is not None:
        model.preprocess_model.coder_groups = args.coder_groups
    if args.no_plans:
        model.use_plans = False
    if args.no_geglu_fuse:
        ops.GEGLU_FUSED = False

    g0 = rank * B  # global image indices of this rank's shard (weak scaling: B per GPU)
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + g0 + i) for i in range(B)])).to(dev)
    draws = [relay_noise((1, 4, S // 8, S // 8), 231 + g0 + i, args.ddim_steps) for i in range(B)]
    noise = torch.cat([d[0] for d in draws])
    step_noise = torch.cat([d[1] for d in draws], 1) if args.sampler == "ddpm" else None
    ctx = synth_context().to(dev)
    mse = torch.empty(B, dtype=torch.float32, device=dev)

    def step():
        out, bodies = model.codec_images(imgs, ctx, noise, steps=args.ddim_steps, sampler=args.sampler,
                                         step_noise_nchw=step_noise)
        ops.call("rdeic_image_mse", imgs.data_ptr(), out.data_ptr(), B, S * S * 3, mse.data_ptr(), ops.stream_ptr())
        m = mse.cpu().numpy()
        rows = torch.tensor([[len(b) * 8.0 / (S * S), float(len(b)),
                              10 * math.log10(255.0 ** 2 / max(float(v), 1e-10)), float(v), 1.0, float(rank)]
                             for b, v in zip(bodies, m)], dtype=torch.float32, device=dev)
        return parallel.gather_metrics(rows)

    for _ in range(args.warmup):
        step()
    if not args.no_roofline:
        # native launch profiler: the launchers record HIP events on their own stream for one launch
        # in --prof-every of each kind (an event pair is two queue markers, i.e. GPU time)
        ops.prof_start(2048 * max(1, args.steps) + 1024, args.prof_every)
    parallel.barrier(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        metrics = step()
    parallel.barrier(dev)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = None
    if not args.no_roofline:
        ops.prof_stop()
        prof = ops.prof_read()
    elapsed = parallel.max_over_ranks(elapsed, dev)
    total_images = B * world * args.steps
    value = total_images / elapsed
    if rank != 0:
        return

    roof = None
    if prof and "conv" in prof:
        n, flops, ms = prof["conv"]
        achieved = flops / (ms * 1e-3) / 1e12
        peak = PEAK_BF16_TFLOPS if dtype == torch.bfloat16 else PEAK_FP32_TFLOPS
        roof = {"bound": "mfma", "kernel": "conv_dma_kernel / conv_kernel (implicit-GEMM conv + linear, rdeic_conv2d)",
                "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": conv_traffic(), "launches_per_step": round(n / args.steps, 1),
                "sampling": f"launches >= 50 GFLOP always timed, smaller ones 1 in {args.prof_every} (weighted)",
                "avg_launch_us": round(ms * 1e3 / max(1, n), 2), "ms_per_step": round(ms / args.steps, 3),
                "kernel_share_of_step": round(ms * 1e-3 / elapsed, 4)}
        # secondary kernels the north star names: attention on MFMA, GroupNorm on HBM
        sec = {}
        for kind, (cnt, work, kms) in prof.items():
            if kind == "conv" or kms <= 0:
                continue
            if kind.startswith("attention"):
                a = work / (kms * 1e-3) / 1e12
                sec[kind] = {"bound": "mfma", "achieved": round(a, 2), "peak": peak, "unit": "TFLOP/s",
                             "frac": round(a / peak, 4), "launches_per_step": round(cnt / args.steps, 1),
                             "ms_per_step": round(kms / args.steps, 3)}
            else:
                a = work / (kms * 1e-3) / 1e9
                sec[kind] = {"bound": "hbm", "achieved": round(a, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                             "frac": round(a / PEAK_HBM_GBS, 4), "launches_per_step": round(cnt / args.steps, 1),
                             "ms_per_step": round(kms / args.steps, 3)}
        roof["secondary"] = sec
    mrows = metrics.cpu().numpy()
    cpu = None
    if not args.no_cpu_baseline:
        try:
            from oracle.bench_cpu import run_cpu_baseline
            cpu = run_cpu_baseline(size=S, steps=args.ddim_steps, rate_gain=rate_gain)
        except Exception as e:  # the baseline is reported, never the target
            cpu = {"value": None, "error": f"{type(e).__name__}: {e}"}
    cfg_name = {(512, 2): "config 2", (1024, 5): "config 3"}.get((S, args.ddim_steps), "custom")
    line = {
        "metric": f"{S}x{S} images/sec encode+relay-decode @ fixed bpp (bitstream-parity path); 1/2/4/8 GPU",
        "value": round(value, 3), "unit": "images/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded images, random-init weights)",
        "config": {"workload": f"{cfg_name}: batch {B}/GPU {S}x{S}, {args.ddim_steps}-step relay "
                               f"{'DDIM' if args.sampler == 'ddim' else 'spaced DDPM'}, "
                               f"encode+entropy-code+decode+VAE-decode", "global_batch": B * world,
                   "image_size": S, "ddim_steps": args.ddim_steps, "sampler": args.sampler, "parallelism": f"dp{world}", "rate_gain": rate_gain,
                   "mean_bpp": round(float(mrows[:, 0].mean()), 4),
                   "mean_psnr_db": round(float(mrows[:, 2].mean()), 2)},
        "roofline": roof,
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
