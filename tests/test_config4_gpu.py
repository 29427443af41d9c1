"""Config 4's operating points on one GPU (BASELINE.json configs[3]: 512x512 CLIC2020-shaped
synthetic images, bpp sweep {0.04, 0.08, 0.12}; the reference gathers one metrics.csv row per image,
inference_partition.py:563-571). The 8-GPU data-parallel part is the bench's (no data-path
collective; tests/test_parallel_cpu.py covers the uneven shards of G=16 on 3 ranks).

Per sweep point (the synthetic rate gain from weights.rate_gain_for_bpp, calibrated on the CPU
oracle), at config 2's batch of 16 bf16 images:
  * the achieved mean bpp is within +-25% of the target (the calibration is fp32 over 4 images;
    the bf16 path's own bpp is printed);
  * coding is batch-invariant (an image coded alone gives the in-batch bytes) and every body
    decodes to its own latents (one body alone == its row of the batched decode);
and at 0.04 and 0.12 one fp32 image's file body is byte-equal to the oracle's compress
(oracle/model_ref.compress restates model/compression.py:151-213 + utils/ckbd.py:76-134) fed the
same VAE feature h (0.08 is test_config2_gpu.py's)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
SIZE = 512
SEEDS = list(range(231, 247))


@pytest.fixture(scope="module")
def imgs():
    from rdeic_amd.synthetic import synth_image
    return torch.from_numpy(np.stack([synth_image(SIZE, SIZE, s) for s in SEEDS])).cuda()


@pytest.mark.parametrize("target", [0.04, 0.08, 0.12])
def test_config4_sweep_point_bf16(gpu, imgs, target):
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    gain = W.rate_gain_for_bpp(target)
    m = RDEIC(compute_dtype=torch.bfloat16).init_synthetic(rate_gain=gain)
    m.preprocess_model.update(force=True)
    with torch.no_grad():
        bodies = m.compress_images(imgs)
        bpp = np.array([8.0 * len(b) / SIZE ** 2 for b in bodies])
        print(f"target {target}: gain {gain}, achieved mean bpp {bpp.mean():.4f} "
              f"(min {bpp.min():.4f}, max {bpp.max():.4f})")
        assert abs(bpp.mean() - target) <= 0.25 * target, bpp.mean()
        for i in (0, 9):
            assert m.compress_images(imgs[i:i + 1])[0] == bodies[i]
        c_b, h_b = m.decompress_bodies(bodies)
        assert bool(torch.isfinite(c_b).all()) and bool(torch.isfinite(h_b.float()).all())
        for i in (3, 15):
            c_s, h_s = m.decompress_bodies(bodies[i:i + 1])
            assert torch.equal(c_b[i:i + 1], c_s) and torch.equal(h_b[i:i + 1], h_s)
    del m
    torch.cuda.empty_cache()


@pytest.mark.parametrize("target", [0.04, 0.12])
def test_config4_sweep_point_fp32_body_vs_oracle(gpu, imgs, target):
    from oracle import model_ref as M
    from rdeic_amd import bitstream
    from rdeic_amd import weights as W
    from rdeic_amd.rdeic import RDEIC
    gain = W.rate_gain_for_bpp(target)
    m = RDEIC(compute_dtype=torch.float32).init_synthetic(rate_gain=gain)
    m.preprocess_model.update(force=True)
    torch.set_num_threads(16)
    with torch.no_grad():
        h = m.encode_images_nhwc(imgs[:1])
        out = m.preprocess_model.compress(h)
        body = bitstream.pack_body(out[0]["shape"], out[0]["strings"])
        sd = M.synthetic_state_dict(rate_gain=gain)
        ref, _, _ = M.compress(sd, h.permute(0, 3, 1, 2).contiguous().cpu(), M.Tables(), coder="c")
    print(f"target {target}: fp32 body {len(body)} B ({8.0 * len(body) / SIZE ** 2:.4f} bpp), oracle {len(ref)} B")
    assert body == ref
    del m
    torch.cuda.empty_cache()
