"""Where does a captured fine-tune step's wall time go? Builds config 5's CapturedStep as bench_train.py does, then
times (a) the host side of graph.replay() (call returns) and (b) the device side (HIP events around the replay) for a
few steps, back to back and one at a time.
usage (GPU box): python tools/graph_replay_probe.py [--dtype bf16] [--steps 5]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    from rdeic_amd.finetune import CapturedStep, FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws
    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    model = RDEIC(compute_dtype=dtype, device=dev).init_synthetic()
    ft = FineTuner(model)
    S = 512
    img = torch.from_numpy(np.stack([synth_image(S, S, 1000)])).to(dev)
    ctx = synth_context().to(dev)
    slice_ch = model.cfg["compression"]["slice_ch"]
    draws = [nchw_draws_to_nhwc(train_draws(1, S // 8, S // 8, slice_ch, s, model.used_timesteps), dev)
             for s in range(args.steps + 3)]
    g = CapturedStep(ft, img, ctx, draws[0])
    for s in range(2):
        g.step(img, draws[s])
    torch.cuda.synchronize()
    # one at a time: host time of step() (copies + replay enqueue), device time between events
    host, devt = [], []
    for s in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        g.step(img, draws[s + 2])
        t1 = time.perf_counter()
        e1.record()
        e1.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e3)
        devt.append(e0.elapsed_time(e1))
        print(f"step {s}: host enqueue {host[-1]:.2f} ms, device {devt[-1]:.2f} ms, wall to completion {(t2 - t0) * 1e3:.2f} ms",
              flush=True)
    # back to back
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        g.step(img, draws[s + 2])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"back to back: {args.steps} steps enqueued in {(t1 - t0) * 1e3:.1f} ms, done after {(t2 - t0) * 1e3:.1f} ms "
          f"({(t2 - t0) * 1e3 / args.steps:.2f} ms/step)", flush=True)


if __name__ == "__main__":
    main()
