"""Probe: wall time of CapturedStep.step vs the eager step at 512^2 B=1 (how much host time the graph removes)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd.finetune import CapturedStep, FineTuner, nchw_draws_to_nhwc  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import synth_context, synth_image, train_draws  # noqa: E402

dt = torch.bfloat16 if (len(sys.argv) > 1 and sys.argv[1] == "bf16") else torch.float32
m = RDEIC(compute_dtype=dt).init_synthetic()
ft = FineTuner(m)
img = torch.from_numpy(synth_image(512, 512, 5)).cuda()[None]
ctx = synth_context().cuda()
dr = nchw_draws_to_nhwc(train_draws(1, 64, 64, m.cfg["compression"]["slice_ch"], 1, 300), "cuda")
for _ in range(2):
    ft.training_step(img, ctx, dr)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    ft.training_step(img, ctx, dr)
torch.cuda.synchronize()
print("eager ms/step", (time.perf_counter() - t) / 3 * 1e3, flush=True)
cs = CapturedStep(ft, img, ctx, dr)
cs.step(img, dr)
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(3):
    cs.step(img, dr)
torch.cuda.synchronize()
print("graph ms/step", (time.perf_counter() - t) / 3 * 1e3, flush=True)
t = time.perf_counter()
cs.graph.replay()
t1 = time.perf_counter()
torch.cuda.synchronize()
print("replay host ms", (t1 - t) * 1e3, "replay total ms", (time.perf_counter() - t) * 1e3, flush=True)
