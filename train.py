"""Adapter fine-tune CLI (the reference's train.py:10-28 with configs/finetune_ood.yaml) on MI355X.

  python train.py --config configs/finetune_ood.yaml [--max-steps N]
  python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py --config ...

One process per GPU (RCCL): every rank trains on its own synthetic batches; gradients of the
control model + compressor are all-reduced in buckets from the backward (FineTuner.enable_ddp).
Weights: random-init synthetic (rdeic_amd/weights.py) or `model.resume` (reference-named state
dict, loaded with safe loaders only). Logs the reference's loss dict (T/loss, T/l_simple, T/l_bpp,
T/q_bpp, T/l_emb, T/l_guide) every log_every_n_steps and saves the trainable parameters (and the
AdamW state) every every_n_train_steps as safetensors.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import yaml

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


EMBED_PROB = "preprocess_model.quantize.embed_prob"


def load_state(path: str):
    """(state dict, metadata) with safe loaders only (safetensors, or torch.load weights_only)."""
    if path.endswith(".safetensors"):
        from safetensors import safe_open
        from safetensors.torch import load_file
        with safe_open(path, "pt") as f:
            meta = f.metadata() or {}
        return load_file(path), meta
    sd = torch.load(path, map_location="cpu", weights_only=True)
    meta = {"global_step": str(sd["global_step"])} if isinstance(sd.get("global_step"), int) else {}
    return sd.get("state_dict", sd), meta


def precision_dtype(precision):
    """The trainer precision of the config: 32 (the reference's finetune_ood.yaml) or bf16. Lightning's
    16 means fp16 autocast, which this path does not implement: refused rather than silently trained
    in another dtype."""
    p = str(precision).lower()
    if p in ("32", "32-true"):
        return torch.float32
    if p in ("bf16", "bf16-mixed", "bf16-true"):
        return torch.bfloat16
    raise SystemExit(f"precision {precision!r} is not supported (32 or bf16; fp16 autocast is not implemented)")


def save_checkpoint(ft, path: str, step: int) -> None:
    from safetensors.torch import save_file
    out = {n: ft.flat[o:o + k].view(ft.m.store.shapes[n]).detach().cpu().contiguous()
           for n, (o, k) in ft.offsets.items()}
    out[EMBED_PROB] = ft.embed_prob.cpu()
    out["optimizer.exp_avg"] = ft.exp_avg.cpu()
    out["optimizer.exp_avg_sq"] = ft.exp_avg_sq.cpu()
    save_file(out, path, metadata={"global_step": str(step)})


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default=os.path.join(ROOT, "configs", "finetune_ood.yaml"))
    ap.add_argument("--max-steps", type=int, default=None)
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture of the step (one GPU)")
    args = ap.parse_args(argv)
    with open(args.config) as f:
        cfg = yaml.safe_load(f)
    from rdeic_amd import parallel
    from rdeic_amd.finetune import CapturedStep, FineTuneConfig, FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws

    rank, world, local = parallel.init_from_env()
    dev = torch.device("cuda", local)
    mc, dc, lc = cfg["model"], cfg["data"], cfg["lightning"]
    dtype = precision_dtype(mc.get("precision", 32))
    seed = int(lc.get("seed", 231))
    if not mc.get("sd_locked", True) or mc.get("is_refine", False):
        raise SystemExit("only the light adaptation (sd_locked: true, is_refine: false) is supported")
    model = RDEIC(compute_dtype=dtype, device=dev).init_synthetic()
    sd, meta = (load_state(mc["resume"]) if mc.get("resume") else ({}, {}))
    if sd:
        model.load_state_dict(sd, strict=False)
    # the codebook-usage EMA travels with the weights (reference checkpoints and ours)
    ft = FineTuner(model, FineTuneConfig(learning_rate=float(mc["learning_rate"]),
                                         l_guide_weight=float(mc["l_guide_weight"]),
                                         l_bpp_weight=float(mc["l_bpp_weight"]),
                                         used_timesteps=int(mc["used_timesteps"])),
                   embed_prob=sd.get(EMBED_PROB))
    start = 0
    if "optimizer.exp_avg" in sd:  # one of train.py's own checkpoints: continue that run exactly
        start = int(meta.get("global_step", 0))
        ft.load_optimizer_state(sd["optimizer.exp_avg"], sd["optimizer.exp_avg_sq"], start)
    if world > 1:
        ft.enable_ddp()
    S, B = int(dc["out_size"]), int(dc["batch_size"])
    n_img = int(dc.get("n_images", 64))
    pool = torch.from_numpy(np.stack([synth_image(S, S, seed + 1000 * rank + i) for i in range(n_img)])).to(dev)
    ctx = synth_context().to(dev)
    tr = lc["trainer"]
    max_steps = args.max_steps if args.max_steps is not None else int(tr["max_steps"])
    log_every = int(tr.get("log_every_n_steps", 50))
    ck = lc.get("checkpoint", {})
    ck_every = int(ck.get("every_n_train_steps", 0))
    ck_dir = ck.get("dirpath", "./logs/ood_finetune")
    slice_ch = model.cfg["compression"]["slice_ch"]
    rng = np.random.default_rng(seed + rank)
    for _ in range(start):  # the batches the interrupted run already drew
        rng.integers(0, n_img, size=B)
    graph = None
    records = []
    t0 = time.perf_counter()
    for step in range(start + 1, max_steps + 1):
        idx = rng.integers(0, n_img, size=B)
        dr = nchw_draws_to_nhwc(train_draws(B, S // 8, S // 8, slice_ch, seed * 1000003 + step * 131 + rank,
                                            ft.cfg.used_timesteps), dev)
        batch = pool[torch.from_numpy(idx).to(dev)]
        if world == 1 and not args.eager and graph is None:
            graph = CapturedStep(ft, batch, ctx, dr)  # one GPU: the step replays as one hipGraph
        d = graph.step(batch, dr) if graph is not None else ft.training_step(batch, ctx, dr)
        if rank == 0 and (step % log_every == 0 or step == max_steps):
            rec = {k: round(float(v), 6) for k, v in d.items()}
            rec.update(global_step=step, it_per_s=round((step - start) / (time.perf_counter() - t0), 4))
            records.append(rec)
            print(json.dumps(rec), flush=True)
        if rank == 0 and ck_every and step % ck_every == 0:
            os.makedirs(ck_dir, exist_ok=True)
            save_checkpoint(ft, os.path.join(ck_dir, f"ood_finetune_step={step}.safetensors"), step)
    parallel.finish()
    return records


if __name__ == "__main__":
    main()
