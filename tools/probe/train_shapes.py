"""Per-shape timing of the fine-tune step's GEMM and conv launches (one eager bf16 step, 512x512).

Records every autograd.gemm / ops.conv2d call of one step (arguments kept alive), then replays each
call 5x back to back between HIP events (isolated device time, warm L2) and prints the shapes that
cost the most per step, with their TFLOP/s.   python tools/probe/train_shapes.py [--dtype bf16]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    from rdeic_amd import autograd as AG, ops
    from rdeic_amd.finetune import FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws

    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    model = RDEIC(compute_dtype=dtype, device=dev).init_synthetic()
    ft = FineTuner(model)
    img = torch.from_numpy(synth_image(512, 512, 1000)[None]).to(dev)
    ctx = synth_context().to(dev)
    draws = nchw_draws_to_nhwc(train_draws(1, 64, 64, model.cfg["compression"]["slice_ch"], 3,
                                           model.used_timesteps), dev)
    recs = []
    orig_gemm, orig_conv = AG.gemm, ops.conv2d

    def gemm(a, a_off, a_sm, a_sk, b, b_off, b_sk, b_sn, c, c_off, c_sm, *, m, n, k, batch=1, nb2=1, ksplit=0,
             **kw):
        call = (orig_gemm, (a, a_off, a_sm, a_sk, b, b_off, b_sk, b_sn, c, c_off, c_sm),
                dict(m=m, n=n, k=k, batch=batch, nb2=nb2, ksplit=ksplit, **kw))
        call[0](*call[1], **call[2])
        kk = k if ksplit > 0 else k * (batch // nb2)
        fl = 2.0 * m * n * kk * nb2
        lay = ("T" if a_sk == 1 else "N") + ("T" if b_sk == 1 else "N")
        recs.append((f"gemm m{m} n{n} k{k} b{batch} ks{ksplit} {lay}", fl, call))

    def conv2d(x, p, **kw):
        out = orig_conv(x, p, **kw)
        kw2 = dict(kw)
        kw2["out"] = out
        x2 = kw.get("x2")
        ho, wo = out.shape[1], out.shape[2]
        if kw.get("pixel_shuffle"):
            ho, wo = ho // 2, wo // 2
        fl = 2.0 * x.shape[0] * ho * wo * p.cout * p.cin * p.kh * p.kw
        recs.append((f"conv {x.shape[0]}x{x.shape[1]}x{x.shape[2]} {p.cin}->{p.cout} k{p.kh} s{p.stride}"
                     f"{' up2' if kw.get('up2') else ''}", fl, (orig_conv, (x, p), kw2)))
        return out

    AG.gemm, ops.conv2d = gemm, conv2d
    for _ in range(2):
        recs.clear()
        ft.training_step(img, ctx, draws)
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    AG.gemm, ops.conv2d = orig_gemm, orig_conv
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    sk = ops.splitk_allowed()  # as inside training_step
    sk.__enter__()
    for key, fl, (fn, a_, kw_) in recs:
        fn(*a_, **kw_)
        e0.record()
        for _ in range(5):
            fn(*a_, **kw_)
        e1.record()
        e1.synchronize()
        a = agg[key]
        a[0] += 1
        a[1] += fl
        a[2] += e0.elapsed_time(e1) / 5
    tot = collections.defaultdict(lambda: [0.0, 0.0])
    for key, (n, fl, ms) in agg.items():
        t = tot[key.split()[0]]
        t[0] += fl
        t[1] += ms
    for fam, (fl, ms) in tot.items():
        print(f"{fam}: {ms:.2f} ms  {fl / ms / 1e9:.1f} TF/s")
    for key, (n, fl, ms) in sorted(agg.items(), key=lambda kv: -kv[1][2])[:args.top]:
        print(f"{ms:8.3f} ms  x{n:3d}  {fl / ms / 1e9:7.1f} TF/s  {key}")


if __name__ == "__main__":
    main()
