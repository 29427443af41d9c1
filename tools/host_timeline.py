"""Host-side timeline of one bench step (diagnostics): wall time of the host coder calls and of
the plan regions, to attribute the GPU-idle gaps of the rocprof trace."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import coders, compression, plan  # noqa: E402
from rdeic_amd import weights as W  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import relay_noise, synth_context, synth_image  # noqa: E402

EV = []


def wrap(mod, name):
    f = getattr(mod, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        EV.append((name, t0, time.perf_counter()))
        return r
    setattr(mod, name, g)


for n in ("rans_encode_batch", "rans_decode_batch", "ac_encode_uniform", "ac_decode_uniform"):
    wrap(coders, n)
wrap(torch.cuda.Event, "synchronize")


def main():
    B, S = 16, 512
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
    m.preprocess_model.update(force=True)
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
    noise = torch.cat([relay_noise((1, 4, S // 8, S // 8), 231 + i, 2)[0] for i in range(B)])
    ctx = synth_context().cuda()
    for _ in range(3):
        m.codec_images(imgs, ctx, noise, steps=2)
    torch.cuda.synchronize()
    for it in range(2):
        EV.clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bodies = m.compress_images(imgs)
        t1 = time.perf_counter()
        c_lat, hint = m.decompress_bodies(bodies)
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        agg = {}
        for n, a, b in EV:
            v = agg.setdefault(n, [0, 0.0])
            v[0] += 1
            v[1] += (b - a) * 1e3
        print(f"iter {it}: compress {1e3 * (t1 - t0):.2f} ms, decompress (host return) {1e3 * (t2 - t1):.2f} ms, "
              f"sync {1e3 * (t3 - t2):.2f} ms", flush=True)
        for n, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"   {n:22s} x{c:3d} {ms:8.2f} ms", flush=True)
        enc = [(a - t0, b - a) for n, a, b in EV if n == "rans_encode_batch"]
        syn = [(a - t0, b - a) for n, a, b in EV if n == "synchronize"]
        print("   encode at/dur ms", [(round(1e3 * a, 2), round(1e3 * d, 2)) for a, d in enc], flush=True)
        print("   first syncs at/dur ms", [(round(1e3 * a, 2), round(1e3 * d, 2)) for a, d in syn[:4]], flush=True)


if __name__ == "__main__":
    main()
