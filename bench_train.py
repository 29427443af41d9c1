"""Config 5: the adapter fine-tune step (train.py + configs/finetune_ood.yaml, UNet frozen) on N MI355X.

One step = one batch of B synthetic 512x512 OOD-satellite-shaped images per GPU through
  VAE encode (no grad) -> Compression.forward (training: noise likelihoods, VQ contrastive loss)
  -> p_losses (q_sample, NoiseEstimator = control + frozen SD-2.1 UNet) -> backward through the
  frozen UNet into the control model and the compressor -> bucketed gradient all-reduce of the
  76.7M trainable parameters (RCCL, overlapped with the backward) -> AdamW
with the reference's precision (fp32, finetune_ood.yaml `precision: 32`) by default.

  python bench_train.py [--gpus N] [--steps K] [--warmup W] [--batch 1] [--size 512] [--dtype fp32|bf16]
For N > 1 run it as is (it starts N ranks itself, rdeic_amd/launch.py) or under torch.distributed.run
(WORLD_SIZE must equal --gpus); one process per GPU, RCCL. Prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK = {"bf16": 2500.0, "fp32": 157.3}  # dense MFMA TFLOP/s (MI355X_MICROARCH.md)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1, help="images per GPU per step (finetune data_loader batch_size 1)")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--bucket-mb", type=int, default=32)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--conv-option", action="append", default=[], metavar="KEY=VALUE",
                    help="rdeic_set_conv_option(KEY, VALUE) before the run (A/B only)")
    ap.add_argument("--splitk-train", default=None, metavar="KDIV,MAX,TARGET",
                    help="split counts of the step's >= 32 k-tile convs (A/B; ops.SPLITK_TRAIN)")
    ap.add_argument("--ft-splitk", default="short", choices=["short", "long", "off"],
                    help="split-K policy of the step's convs (A/B; finetune.FT_SPLITK)")
    ap.add_argument("--eager", action="store_true",
                    help="eager steps (default on one GPU: the step captured once as a hipGraph and replayed)")
    return ap.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    from rdeic_amd.launch import maybe_launch
    maybe_launch(args.gpus, __file__, sys.argv[1:] if argv is None else list(argv))
    from rdeic_amd import ops, parallel
    from rdeic_amd import finetune
    from rdeic_amd.finetune import CapturedStep, FineTuner, nchw_draws_to_nhwc
    finetune.FT_SPLITK = args.ft_splitk
    for kv in args.conv_option:
        k, v = kv.split("=")
        ops.set_conv_option(int(k), int(v))
    if args.splitk_train:
        ops.SPLITK_TRAIN = tuple(int(v) for v in args.splitk_train.split(","))
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws

    rank, world, local = parallel.init_from_env()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    S, B = args.size, args.batch
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    def log(msg):
        if rank == 0:
            print(f"[bench_train] {msg}", file=sys.stderr, flush=True)

    model = RDEIC(compute_dtype=dtype, device=dev).init_synthetic()
    ft = FineTuner(model)
    if world > 1:
        ft.enable_ddp(bucket_bytes=args.bucket_mb << 20)
    log(f"{ft.num_params() / 1e6:.2f}M trainable parameters, world {world}, batch {B}/GPU, {S}x{S}, {args.dtype}")
    n_img = 4
    pool = torch.from_numpy(np.stack([synth_image(S, S, 1000 + 97 * rank + i) for i in range(n_img)])).to(dev)
    ctx = synth_context().to(dev)
    slice_ch = model.cfg["compression"]["slice_ch"]
    total = args.warmup + args.steps + 1
    draws = [nchw_draws_to_nhwc(train_draws(B, S // 8, S // 8, slice_ch, 7919 * rank + s, model.used_timesteps), dev)
             for s in range(total)]

    def batch(s):
        idx = [(s * B + j) % n_img for j in range(B)]
        return pool[idx]

    losses = []
    graph = None
    if world == 1 and not args.eager:
        graph = CapturedStep(ft, batch(0), ctx, draws[0])
        log("step captured as one hipGraph")

    def step(s):
        if graph is not None:
            return graph.step(batch(s), draws[s])
        return ft.training_step(batch(s), ctx, draws[s])

    for s in range(args.warmup):
        d = step(s)
        torch.cuda.synchronize()
        log(f"warmup step {s}: loss {float(d['T/loss']):.4f}")
    parallel.barrier(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        d = step(args.warmup + s)
        losses.append(d["T/loss"].detach().clone())
    torch.cuda.synchronize()
    parallel.barrier(dev)
    elapsed = parallel.max_over_ranks(time.perf_counter() - t0, dev)
    loss_vals = [float(v) for v in losses]
    ms = 1000.0 * elapsed / args.steps
    log(f"timed {args.steps} steps: {ms:.1f} ms/step, losses {['%.4f' % v for v in loss_vals]}")

    roof = None
    if not args.no_roofline and rank == 0:
        ops.prof_start(65536, 1)
        torch.cuda.synchronize()
        w0 = time.perf_counter()
        ft.training_step(batch(0), ctx, draws[-1])  # eager: the launchers' own events time each kernel
        torch.cuda.synchronize()
        wall = time.perf_counter() - w0
        ops.prof_stop()
        pr = ops.prof_read()
        peak = PEAK[args.dtype]
        fam = {}
        for kind in ("conv", "gemm", "gn_apply"):
            if kind in pr:
                n, work, kms = pr[kind]
                fam[kind] = {"launches": n, "ms": round(kms, 3),
                             ("tflops" if kind != "gn_apply" else "gbs"):
                                 round(work / (kms * 1e-3) / (1e12 if kind != "gn_apply" else 1e9), 2)}
        conv = pr.get("conv")
        gemm = pr.get("gemm")
        fl = (conv[1] if conv else 0.0) + (gemm[1] if gemm else 0.0)
        kms = (conv[2] if conv else 0.0) + (gemm[2] if gemm else 0.0)
        achieved = fl / (kms * 1e-3) / 1e12 if kms else 0.0
        roof = {"bound": "mfma", "kernel": "conv (forward / input-gradient implicit GEMM) + strided GEMM (weight "
                "gradients, attention)", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": None, "flops_per_step": fl,
                "kernel_ms_per_step": round(kms, 3), "step_wall_ms_profiled": round(1000 * wall, 2),
                "families": fam}
    if rank == 0:
        line = {
            "metric": "adapter fine-tune (config 5) 512x512 images/s, UNet frozen, grad all-reduce; 1/2/4/8 GPU",
            "value": round(world * B * args.steps / elapsed, 3),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (seeded OOD-satellite-shaped images, random-init weights, seeded draws)",
            "config": {"workload": "config 5: adapter fine-tune step (control model + compressor trained, SD-2.1 "
                                   "UNet and VAE frozen), AdamW lr 2e-5",
                       "global_batch": world * B, "image_size": S, "parallelism": f"dp{world}",
                       "trainable_params": ft.num_params(), "steps_per_s": round(args.steps / elapsed, 4),
                       "execution": "hipGraph replay of the captured step" if graph is not None else "eager",
                       "mean_loss": round(sum(loss_vals) / len(loss_vals), 5)},
            "roofline": roof,
            "cpu_baseline": None,
        }
        print(json.dumps(line), flush=True)
    parallel.finish()


if __name__ == "__main__":
    main()
