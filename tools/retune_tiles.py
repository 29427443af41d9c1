"""Re-time selected entries of the committed conv tile table against new candidate tiles, on the
layers the bench workloads really run (same driver as tools/tune_tiles.py: config 2, config 3 and
the 128^2 test shapes, eager). An entry is switched only when a candidate beats the table's tile by
more than --margin on the median of interleaved rounds; every tile is bit-identical
(tests/test_tiles_gpu.py), so this changes speed only.

  python tools/retune_tiles.py --cand 37,38 --cout-mult 160 [--configs 16x512x2,...] [--write]
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


class KeyTrack(dict):
    last = None

    def get(self, k, default=None):
        KeyTrack.last = k
        return super().get(k, default)

    def __contains__(self, k):
        KeyTrack.last = k
        return super().__contains__(k)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="16x512x2,8x1024x5,2x128x2")
    ap.add_argument("--cand", default="37,38")
    ap.add_argument("--cout-mult", type=int, default=160)
    ap.add_argument("--margin", type=float, default=0.02)
    ap.add_argument("--write", action="store_true")
    args = ap.parse_args()
    from rdeic_amd import _lib, ops
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import relay_noise, synth_context, synth_image

    cands = [int(c) for c in args.cand.split(",")]
    table = dict(ops.TILE_TABLE)
    done, changes = {}, {}

    def parse(key):
        return int(key.split(":")[2][1:])  # output channels

    def retune(d0, scratch, candidates=None):
        key = KeyTrack.last
        old = table.get(key, -1)
        if key in done or _lib.RECORDER is not None or old < 20 or parse(key) % args.cout_mult:
            return old
        d = ops.ConvDesc.from_buffer_copy(d0)
        d.out = scratch.data_ptr()
        s = ops.stream_ptr()
        tiles = [old] + [c for c in cands if c != old]
        times = {t: [] for t in tiles}
        for t in tiles:
            ops.call("rdeic_conv2d_tile", ops.C.byref(d), t, s)
        for _ in range(5):
            for t in tiles:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    ops.call("rdeic_conv2d_tile", ops.C.byref(d), t, s)
                e1.record()
                e1.synchronize()
                times[t].append(e0.elapsed_time(e1) / 3)
        med = {t: sorted(v)[len(v) // 2] for t, v in times.items()}
        best = min(med, key=med.get)
        pick = best if med[best] < med[old] * (1 - args.margin) else old
        done[key] = pick
        print(json.dumps({"key": key, "old": old, "pick": pick, "us": {t: round(v * 1e3, 1) for t, v in med.items()}}),
              flush=True)
        if pick != old:
            changes[key] = (old, pick)
        return old  # keep running the committed choice during the sweep

    ops._autotune_tile = retune
    ops.AUTOTUNE = True
    # every key must take the autotune path: hide the table from the membership test, keep .get()
    class Hidden(KeyTrack):
        def __contains__(self, k):
            KeyTrack.last = k
            return False
    ops.TILE_TABLE = Hidden(table)

    ctx = synth_context().cuda()
    model = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
    model.preprocess_model.update(force=True)
    for cfg in args.configs.split(","):
        B, S, steps = (int(v) for v in cfg.split("x"))
        imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
        noise = torch.cat([relay_noise((1, 4, S // 8, S // 8), 231 + i, steps)[0] for i in range(B)])
        model.use_plans = False
        model.codec_images(imgs, ctx, noise, steps=steps)
        torch.cuda.synchronize()
        del imgs, noise
        torch.cuda.empty_cache()
    print(json.dumps({"changes": changes}), flush=True)
    if args.write and changes:
        path = os.path.join(ROOT, "rdeic_amd", "conv_tiles.json")
        with open(path) as f:
            tab = json.load(f)
        for k, (_, new) in changes.items():
            tab["tiles"][k] = new
        with open(path, "w") as f:
            json.dump(tab, f, indent=0)
            f.write("\n")


if __name__ == "__main__":
    main()
