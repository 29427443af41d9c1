"""Repeat config 3's B=8 1024^2 bf16 compress (plan replay) and locate any run-to-run difference:
device symbols / indexes (the pinned copies the host coder reads), VQ indexes, or the host coder's
bytes from identical symbols."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from rdeic_amd import weights as W  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import synth_image  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
R = int(sys.argv[3]) if len(sys.argv) > 3 else 12
imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
pc = m.preprocess_model
runs = []
with torch.no_grad():
    for r in range(R):
        bodies = m.compress_images(imgs)
        cache = pc.__dict__.get("_pin_cache", {})
        sym = cache["enc_sym0"].numpy().copy()
        idx = cache["enc_idx0"].numpy().copy()
        zi = cache["enc_zidx"].numpy().copy()
        runs.append((bodies, sym, idx, zi))
        b0, s0, i0, z0 = runs[0]
        same_b = [a == b for a, b in zip(b0, bodies)]
        n = sym.size // B
        same_s = [bool(np.array_equal(s0[k * n:(k + 1) * n], sym[k * n:(k + 1) * n])) for k in range(B)]
        same_i = [bool(np.array_equal(i0[k * n:(k + 1) * n], idx[k * n:(k + 1) * n])) for k in range(B)]
        print(f"run {r}: bodies {same_b} sym {same_s} idx {same_i} zidx {bool(np.array_equal(z0, zi))}", flush=True)
        if not all(same_s):
            k = same_s.index(False)
            d = np.nonzero(s0[k * n:(k + 1) * n] != sym[k * n:(k + 1) * n])[0]
            print(f"   image {k}: {d.size} symbols differ, first at {d[:8]} of {n}", flush=True)
