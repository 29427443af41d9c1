"""Find the synthetic rate_gain (rdeic_amd/weights.py RATE_LAYERS) that gives a target bpp on the
bench's synthetic 512x512 images, with the CPU oracle (test infrastructure; runs in this container)."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import model_ref as M  # noqa: E402
from rdeic_amd import weights as W  # noqa: E402
from rdeic_amd.synthetic import synth_image  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--images", type=int, default=2)
    ap.add_argument("--gains", default="1,0.3,0.1,0.05,0.03,0.02,0.01")
    args = ap.parse_args()
    torch.set_num_threads(8)
    sd1 = M.synthetic_state_dict()
    tables = M.Tables()
    hs = []
    with torch.no_grad():
        for i in range(args.images):
            img = synth_image(args.size, args.size, 231 + i)
            x = torch.tensor(img[None] / 255.0, dtype=torch.float32).permute(0, 3, 1, 2).contiguous()
            hs.append(M.vae_encode_hc(sd1, x * 2 - 1) * 0.18215)
        for g in [float(v) for v in args.gains.split(",")]:
            sd = M.synthetic_state_dict(rate_gain=g)
            bpps = []
            for h in hs:
                body, sym, _ = M.compress(sd, h, tables, coder="c")
                bpps.append(8.0 * len(body) / (args.size * args.size))
            nz = float((np.asarray(sym) != 0).mean())
            print(f"rate_gain {g:8.4f}  bpp {np.mean(bpps):.4f}  ({', '.join(f'{b:.4f}' for b in bpps)})  "
                  f"nonzero symbols {nz:.4f}", flush=True)


if __name__ == "__main__":
    main()
