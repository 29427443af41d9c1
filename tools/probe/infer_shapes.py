"""Per-layer timing of the config-2 codec step's convs (B=16, 512x512, bf16, 2 DDIM steps).

Runs one step without launch plans, records every ops.conv2d call (arguments kept alive, split-K
state as it was), then replays each call 3x back to back between HIP events and prints the layer
classes that cost the most per step with their TFLOP/s and tile.
    python tools/probe/infer_shapes.py [--batch 16] [--top 50]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--top", type=int, default=50)
    args = ap.parse_args()
    from rdeic_amd import ops
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image

    dev = torch.device("cuda", 0)
    S, B = args.size, args.batch
    model = RDEIC(compute_dtype=torch.bfloat16, device=dev)
    model.use_plans = False
    model.init_synthetic()
    model.preprocess_model.update(force=True)
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + g) for g in range(B)])).to(dev)
    draws = [relay_noise((1, 4, S // 8, S // 8), 231 + g, 2) for g in range(B)]
    noise = torch.cat([d[0] for d in draws])
    ctx = synth_context().to(dev)
    model.codec_images(imgs, ctx, noise, steps=2)
    torch.cuda.synchronize()

    recs = []
    orig = ops.conv2d

    def conv2d(x, p, **kw):
        out = orig(x, p, **kw)
        kw2 = dict(kw)
        kw2["out"] = out
        ho, wo = out.shape[1], out.shape[2]
        if kw.get("pixel_shuffle"):
            ho, wo = ho // 2, wo // 2
        cin = p.cin
        fl = 2.0 * x.shape[0] * ho * wo * p.cout * cin * p.kh * p.kw
        M = x.shape[0] * ho * wo
        key = (f"M{M} {x.shape[1]}x{x.shape[2]} {cin}->{p.cout} k{p.kh} s{p.stride}"
               f"{' up2' if kw.get('up2') else ''}{' gn' if kw.get('gn') is not None else ''}"
               f"{' res' if kw.get('res') is not None else ''}{' geglu' if kw.get('geglu') else ''}")
        recs.append((key, fl, x, p, kw2, ops.SPLITK_ALLOWED))
        return out

    ops.conv2d = conv2d
    model.codec_images(imgs, ctx, noise, steps=2)
    torch.cuda.synchronize()
    ops.conv2d = orig
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for key, fl, x, p, kw, sk in recs:
        prev = ops.SPLITK_ALLOWED
        ops.SPLITK_ALLOWED = sk
        orig(x, p, **kw)
        e0.record()
        for _ in range(3):
            orig(x, p, **kw)
        e1.record()
        e1.synchronize()
        ops.SPLITK_ALLOWED = prev
        a = agg[key]
        a[0] += 1
        a[1] += fl
        a[2] += e0.elapsed_time(e1) / 3
    tf = sum(v[1] for v in agg.values())
    ms = sum(v[2] for v in agg.values())
    print(f"conv total: {len(recs)} calls, {tf / 1e12:.2f} TFLOP, {ms:.2f} ms, {tf / ms / 1e9:.1f} TF/s")
    for key, (n, fl, t) in sorted(agg.items(), key=lambda kv: -kv[1][2])[:args.top]:
        print(f"{t:8.3f} ms  x{n:3d}  {fl / t / 1e9:7.1f} TF/s  {fl / 1e12:6.2f} TF  {key}")


if __name__ == "__main__":
    main()
