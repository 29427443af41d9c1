"""Per-layer time of the bench's conv / linear launches: one eager codec step of config 2 (B = 16, 512^2,
2 DDIM steps, bf16) with ops.conv2d wrapped in HIP events (on the launch stream; includes a materialised
GroupNorm apply and the split-K reduce of the call). Grouped by layer shape, sorted by time: ms per step,
algorithmic TFLOP/s, launches. Tells which layer classes hold the conv family's time.
usage (GPU box): python tools/layer_times.py [--size 512 --batch 16] > out.txt"""
import argparse
import collections
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import relay_noise, synth_context, synth_image  # noqa: E402

LOG = []
_conv2d = ops.conv2d


def timed(x, p, **kw):
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    out = _conv2d(x, p, **kw)
    e1.record()
    x2 = kw.get("x2")
    cin = x.shape[3] + (x2.shape[3] if x2 is not None else 0)
    key = (x.shape[0], x.shape[1], x.shape[2], cin, p.cout, p.kh, p.stride, int(kw.get("up2", False)),
           int(kw.get("gn") is not None), int(kw.get("res") is not None), int(kw.get("geglu", False)),
           int(kw.get("pixel_shuffle", False)), int(kw.get("ln_rows") is not None))
    ho, wo = out.shape[1], out.shape[2]
    if kw.get("pixel_shuffle"):
        ho, wo = ho // 2, wo // 2
    flops = 2.0 * out.shape[0] * ho * wo * p.cout * p.kh * p.kw * p.cin
    LOG.append((key, flops, e0, e1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    S, B = a.size, a.batch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = RDEIC(compute_dtype=torch.bfloat16, device=dev)
    model.use_plans = False
    model.init_synthetic()
    model.preprocess_model.update(force=True)
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + g) for g in range(B)])).to(dev)
    draws = [relay_noise((1, 4, S // 8, S // 8), 231 + g, a.steps) for g in range(B)]
    noise = torch.cat([d[0] for d in draws])
    ctx = synth_context().to(dev)
    model.codec_images(imgs, ctx, noise, steps=a.steps, sampler="ddim")  # warm-up
    torch.cuda.synchronize()
    ops.conv2d = timed
    try:
        model.codec_images(imgs, ctx, noise, steps=a.steps, sampler="ddim")
        torch.cuda.synchronize()
    finally:
        ops.conv2d = _conv2d
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for key, fl, e0, e1 in LOG:
        r = agg[key]
        r[0] += 1
        r[1] += fl
        r[2] += e0.elapsed_time(e1)
    rows = sorted(agg.items(), key=lambda kv: -kv[1][2])
    tot_ms = sum(v[2] for v in agg.values())
    tot_fl = sum(v[1] for v in agg.values())
    print(f"# conv calls {len(LOG)}, {tot_ms:.2f} ms, {tot_fl / 1e12:.2f} TFLOP, {tot_fl / tot_ms / 1e9:.0f} TF")
    print("# key = (n, h, w, cin, cout, k, stride, up2, gn_in, res, geglu, pixel_shuffle, ln_fold)")
    for key, (n, fl, ms) in rows:
        print(f"{ms:9.3f} ms {fl / ms / 1e9:8.1f} TF x{n:4d}  {key}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"total_ms": tot_ms, "total_tflop": tot_fl / 1e12,
                       "layers": [{"key": list(k), "launches": v[0], "ms": round(v[2], 4),
                                   "tflops": round(v[1] / v[2] / 1e9, 1)} for k, v in rows]}, f, indent=0)


if __name__ == "__main__":
    main()
