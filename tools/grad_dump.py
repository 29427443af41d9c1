"""Dump the fp32 fine-tune step's gradients (norm + the 4 seeded projections of every trainable tensor) at 128^2
and 512^2, exactly as tests/test_finetune_gpu.py's fixture computes them, for the offline comparison against the
reference's fp32 golden (train_{size}.npz) and its float64 twin (train_{size}_f64.npz).
usage (GPU box): python tools/grad_dump.py OUT_DIR"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rdeic_amd.finetune import FineTuner, nchw_draws_to_nhwc
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_context, synth_image, train_draws
    from tests.golden.train_proj import projections
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    for size in (128, 512):
        m = RDEIC(compute_dtype=torch.float32).init_synthetic()
        ft = FineTuner(m)
        dr = train_draws(1, size // 8, size // 8, m.cfg["compression"]["slice_ch"], 5, m.used_timesteps)
        img = torch.from_numpy(synth_image(size, size, 231)).cuda()[None]
        ctx = synth_context().cuda()
        d = nchw_draws_to_nhwc(dr, "cuda")
        ft.zero_grad()
        x_start, h = ft.get_first_stage(img, d["post_eps"])
        loss, ld = ft.losses(x_start, h, ctx, d["t"], d["noise"], d["slice_noise"])
        loss.backward()
        torch.cuda.synchronize()
        names, norms, projs = [], [], []
        for n, (o, k) in ft.offsets.items():
            g = ft.grad[o:o + k].cpu()
            names.append(n)
            norms.append(float(g.double().norm()))
            projs.append(projections(n, g))
        np.savez(os.path.join(out, f"grads_{size}.npz"), grad_names=np.asarray(names), grad_norm=np.asarray(norms),
                 grad_proj=np.stack(projs))
        print(size, "dumped", len(names), flush=True)
        del ft, m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
