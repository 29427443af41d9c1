"""Per-stage and per-conv-class timing of the bench workload (diagnostics, not the bench)."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import sampler_noise, synth_context, synth_image  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    r = fn()
    torch.cuda.synchronize()
    return r, (time.perf_counter() - t) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--paths", default="2")
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    B, S = args.batch, args.size
    model = RDEIC(compute_dtype=torch.bfloat16).init_synthetic()
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
    noise = torch.cat([sampler_noise((1, 4, S // 8, S // 8), 231 + i)[1] for i in range(B)])
    ctx = synth_context().cuda()
    for path in [int(p) for p in args.paths.split(",")]:
        ops.set_conv_path(path)
        model.codec_images(imgs, ctx, noise, steps=2)  # warmup
        stages = {}
        marks = {}
        ops.PROFILE = []

        def timed_stage(name, fn):
            n0 = len(ops.PROFILE)
            r, stages[name] = timed(fn)
            marks[name] = (n0, len(ops.PROFILE))
            return r

        h = timed_stage("encode_vae", lambda: model.encode_images_nhwc(imgs))
        outs = timed_stage("compress_nets+coder", lambda: model.preprocess_model.compress(h))
        from rdeic_amd import bitstream
        bodies = [bitstream.pack_body(o["shape"], o["strings"]) for o in outs]
        c_lat, hint = timed_stage("decompress", lambda: model.decompress_bodies(bodies))
        nz = ops.nchw_to_nhwc(noise.cuda(), torch.float32)
        z = timed_stage("relay_sample_2steps", lambda: model.relay_sample_nhwc(c_lat, hint, ctx, nz, 2))
        x = timed_stage("vae_decode", lambda: model.decode_nhwc(z))
        timed_stage("to_u8", lambda: model.to_image_u8(x))
        torch.cuda.synchronize()
        prof, ops.PROFILE = ops.PROFILE, None
        n, flops, ms = ops.conv_profile_summary(prof)
        conv_stage = {}
        for k, (a0, a1) in marks.items():
            _, f, m = ops.conv_profile_summary(prof[a0:a1]) if a1 > a0 else (0, 0.0, 0.0)
            conv_stage[k] = round(m, 2)
        print(json.dumps({"conv_path": path, "stages_ms": {k: round(v, 2) for k, v in stages.items()},
                          "conv_ms_by_stage": conv_stage,
                          "total_ms": round(sum(stages.values()), 2), "conv_launches": n,
                          "conv_ms": round(ms, 2), "conv_tflops": round(flops / ms / 1e9, 1)}), flush=True)
        bd = ops.conv_profile_breakdown(prof)
        for k, (cnt, gf, t) in sorted(bd.items(), key=lambda kv: -kv[1][2])[:args.top]:
            print(f"  {t:8.2f} ms  {gf / t:7.1f} TF  x{cnt:3d}  {k}", flush=True)
    ops.set_conv_path(2)


if __name__ == "__main__":
    main()
