"""Measure the per-shape conv tile table (rdeic_amd/conv_tiles.json) on one MI355X.

Runs the bench workloads (config 2: B=16 512^2, 2-step relay; config 3: B=8 1024^2, 5 steps; the
128^2 test shapes) once with ops.AUTOTUNE on, so every bf16 big-tile conv shape on the path times
its candidate tiles, and writes the winners. All tiles give bit-identical results
(tests/test_tiles_gpu.py), so the table only fixes WHICH kernel runs per shape — deterministically,
in every process and on every box.

  python tools/tune_tiles.py [--configs 16x512x2,8x1024x5,2x128x2] [--out rdeic_amd/conv_tiles.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="16x512x2,8x1024x5,2x128x2")
    ap.add_argument("--out", default=os.path.join(ROOT, "rdeic_amd", "conv_tiles.json"))
    ap.add_argument("--fresh", action="store_true", help="ignore the existing table (re-time every shape)")
    args = ap.parse_args()
    from rdeic_amd import ops
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image

    if args.fresh:
        ops.TILE_TABLE.clear()
    ops.AUTOTUNE = True
    ctx = synth_context().cuda()
    model = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
    model.preprocess_model.update(force=True)
    for cfg in args.configs.split(","):
        B, S, steps = (int(v) for v in cfg.split("x"))
        n0 = len(ops.TILE_TABLE)
        imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
        noise = torch.cat([relay_noise((1, 4, S // 8, S // 8), 231 + i, steps)[0] for i in range(B)])
        model.use_plans = False  # eager: every conv goes through ops.conv2d (plans do not re-tune)
        model.codec_images(imgs, ctx, noise, steps=steps)
        torch.cuda.synchronize()
        print(f"{cfg}: {len(ops.TILE_TABLE) - n0} new shapes", flush=True)
        del imgs, noise
        torch.cuda.empty_cache()
    with open(args.out, "w") as f:
        json.dump({"source": "tools/tune_tiles.py on one MI355X (gfx950); per-shape fastest of the candidate "
                             "tiles, every tile bit-identical", "tiles": dict(sorted(ops.TILE_TABLE.items()))},
                  f, indent=0)
    print(f"wrote {len(ops.TILE_TABLE)} shapes to {args.out}")


if __name__ == "__main__":
    main()
