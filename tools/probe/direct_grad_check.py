"""How many trainable parameters take the direct-gradient path in one fine-tune step (128^2 fp32),
and which torch elementwise kernels remain (profiler op counts)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import autograd as AG, ops  # noqa: E402
from rdeic_amd.finetune import FineTuner, nchw_draws_to_nhwc  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import synth_context, synth_image, train_draws  # noqa: E402

dt = torch.bfloat16 if len(sys.argv) > 1 and sys.argv[1] == "bf16" else torch.float32
m = RDEIC(compute_dtype=dt).init_synthetic()
ft = FineTuner(m)
d = nchw_draws_to_nhwc(train_draws(1, 16, 16, m.cfg["compression"]["slice_ch"], 5, m.used_timesteps), "cuda")
img = torch.from_numpy(synth_image(128, 128, 231)).cuda()[None]
ctx = synth_context().cuda()
ft.zero_grad()
x_start, h = ft.get_first_stage(img, d["post_eps"])
with ops.splitk_allowed():
    loss, _ = ft.losses(x_start, h, ctx, d["t"], d["noise"], d["slice_noise"])
    counted = [n for n in ft.offsets if getattr(ft.p(n), "_rdeic_uses", 0) > 0]
    print("params", len(ft.offsets), "counted for direct grads", len(counted))
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
        loss.backward()
left = [n for n in counted if ft.p(n)._rdeic_uses != 0]
print("still pending after backward", len(left), left[:5])
print(prof.key_averages().table(sort_by="count", row_limit=25))
