"""Throughput of the config-2 codec with 1 vs 2 concurrent sessions (host thread + HIP stream each)."""
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import weights as W  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import relay_noise, synth_context, synth_image  # noqa: E402


def main():
    B, S, K = 16, 512, 8
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=W.RATE_GAIN_BPP008)
    m.preprocess_model.update(force=True)
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + i) for i in range(B)])).cuda()
    noise = torch.cat([relay_noise((1, 4, S // 8, S // 8), 231 + i, 2)[0] for i in range(B)])
    ctx = synth_context().cuda()
    sess = [m, m.session(), m.session()]
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = {}
    for i, (s, st) in enumerate(zip(sess, streams)):  # record plans one session at a time
        with torch.cuda.stream(st):
            for _ in range(2):
                outs[i] = s.codec_images(imgs, ctx, noise, steps=2)
        torch.cuda.synchronize()
    for ns in (1, 2, 3):

        def work(i, n):
            with torch.cuda.stream(streams[i]):
                for _ in range(n):
                    o, b = sess[i].codec_images(imgs, ctx, noise, steps=2)
                torch.cuda.current_stream().synchronize()
                outs[i] = (o, b)

        torch.cuda.synchronize()
        t0 = time.perf_counter()
        th = [threading.Thread(target=work, args=(i, K // ns)) for i in range(ns)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        same = all(outs[i][1] == outs[0][1] and torch.equal(outs[i][0], outs[0][0]) for i in range(ns))
        print(f"sessions {ns}: {B * (K // ns) * ns / dt:.1f} img/s  (identical outputs across sessions: {same})",
              flush=True)


if __name__ == "__main__":
    main()
