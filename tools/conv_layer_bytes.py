"""Per-layer algorithmic bytes of the bench's conv / linear launches: one eager
codec step of config 2 (B = 16, 512^2, 2 DDIM steps, bf16) with ops.conv2d wrapped to log each call's
shape. Bytes per call follow the library's own count (conv_gemm.hip conv_bytes, RDEIC_PROF_CONV_BYTES):
input once + packed weights once + output once (+ residual once). Prints a JSON table grouped by layer
shape, sorted by bytes per step, and the step total to compare with the bench line's
roofline.algorithmic_bytes_per_step and the PMC traffic (profiles/*conv_traffic.json).
usage (GPU box): python tools/conv_layer_bytes.py > out.json"""
import collections
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rdeic_amd import ops  # noqa: E402
from rdeic_amd.rdeic import RDEIC  # noqa: E402
from rdeic_amd.synthetic import relay_noise, synth_context, synth_image  # noqa: E402

LOG = []
_conv2d = ops.conv2d


def logged(x, p, **kw):
    out = _conv2d(x, p, **kw)
    x2 = kw.get("x2")
    es = x.element_size()
    cin = x.shape[3] + (x2.shape[3] if x2 is not None else 0)
    n, h, w = x.shape[0], x.shape[1], x.shape[2]
    inb = n * h * w * cin * es
    wb = p.cout * p.kh * p.kw * p.cin * es
    ob = out.numel() * out.element_size()
    rb = ob if kw.get("res") is not None else 0
    key = (n, h, w, cin, p.cout, p.kh, int(kw.get("up2", False)), int(kw.get("gn") is not None),
           int(kw.get("res") is not None), int(kw.get("geglu", False)), int(kw.get("pixel_shuffle", False)))
    LOG.append((key, inb + wb + ob + rb, 2.0 * out.shape[0] * out.shape[1] * out.shape[2] * p.cout
                * p.kh * p.kw * p.cin * (1 if not kw.get("pixel_shuffle") else 0.25)))
    return out


def main():
    S, B = 512, 16
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = RDEIC(compute_dtype=torch.bfloat16, device=dev)
    model.use_plans = False
    model.init_synthetic()
    model.preprocess_model.update(force=True)
    imgs = torch.from_numpy(np.stack([synth_image(S, S, 231 + g) for g in range(B)])).to(dev)
    draws = [relay_noise((1, 4, S // 8, S // 8), 231 + g, 2) for g in range(B)]
    noise = torch.cat([d[0] for d in draws])
    ctx = synth_context().to(dev)
    model.codec_images(imgs, ctx, noise, steps=2, sampler="ddim")  # warm-up (tile table, workspaces)
    torch.cuda.synchronize()
    ops.conv2d = logged
    try:
        model.codec_images(imgs, ctx, noise, steps=2, sampler="ddim")
        torch.cuda.synchronize()
    finally:
        ops.conv2d = _conv2d
    agg = collections.OrderedDict()
    for key, b, f in LOG:
        e = agg.setdefault(key, [0, 0.0, 0.0])
        e[0] += 1
        e[1] += b
        e[2] += f
    rows = [{"layer": dict(zip(("n", "h", "w", "cin", "cout", "k", "up2", "gn_in", "res", "geglu", "pixel_shuffle"), k)),
             "launches": v[0], "algorithmic_mb_per_launch": round(v[1] / v[0] / 1e6, 3),
             "algorithmic_gb_per_step": round(v[1] / 1e9, 4), "gflop_per_step": round(v[2] / 1e9, 1)}
            for k, v in agg.items()]
    rows.sort(key=lambda r: -r["algorithmic_gb_per_step"])
    tot_b = sum(b for _, b, _ in LOG)
    print(json.dumps({"workload": {"size": S, "batch": B, "ddim_steps": 2, "dtype": "bf16", "sampler": "ddim"},
                      "source": "tools/conv_layer_bytes.py: ops.conv2d calls of one eager codec step (Python-level "
                                "count; the library's RDEIC_PROF_CONV_BYTES counts the same terms per launch)",
                      "conv2d_calls": len(LOG), "algorithmic_gb_per_step": round(tot_b / 1e9, 3),
                      "algorithmic_mb_per_call": round(tot_b / len(LOG) / 1e6, 3), "layers": rows}, indent=1))


if __name__ == "__main__":
    main()
