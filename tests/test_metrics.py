"""Image-quality metrics: the CPU restatement (oracle/metrics_ref.py) on its defining properties,
and the device kernels (rdeic_image_ssim, via rdeic_amd/metrics.py) against it. pyiqa — the
reference's metric library — is not installed here: parity with it is unpinned."""
import numpy as np
import pytest
import torch

from oracle import metrics_ref as R


def _pair(seed, size=256, noise=12.0):
    from rdeic_amd.synthetic import synth_image
    a = synth_image(size, size, seed)
    rng = np.random.default_rng(seed)
    b = np.clip(a.astype(np.float64) + rng.normal(0, noise, a.shape), 0, 255).astype(np.uint8)
    return b, a


def test_oracle_metric_properties():
    b, a = _pair(1)
    assert R.ssim_ms_ssim(a, a) == (1.0, 1.0)
    s, ms = R.ssim_ms_ssim(b, a)
    s2, ms2 = R.ssim_ms_ssim(a, b)
    assert 0.0 < s < 1.0 and 0.0 < ms < 1.0
    assert abs(s - s2) < 1e-12 and abs(ms - ms2) < 1e-12  # symmetric
    b2, _ = _pair(1, noise=30.0)
    assert R.ssim_ms_ssim(b2, a)[0] < s  # more noise, lower score
    assert R.psnr(a, a) == 100.0
    assert abs(R.gaussian_2d().sum() - 1.0) < 1e-12


@pytest.mark.gpu
def test_device_ssim_ms_ssim_match_restatement(gpu):
    from rdeic_amd import metrics
    pairs = [_pair(s, size) for s, size in ((3, 256), (4, 256), (5, 256))] + [_pair(6, 512)]
    for size in (256, 512):
        ps = [p for p in pairs if p[0].shape[0] == size]
        pred = torch.from_numpy(np.stack([p[0] for p in ps])).cuda()
        tgt = torch.from_numpy(np.stack([p[1] for p in ps])).cuda()
        ss, ms = metrics.ssim_ms_ssim(pred, tgt)
        pp = metrics.psnr(pred, tgt)
        for i, (b, a) in enumerate(ps):
            rs, rm = R.ssim_ms_ssim(b, a)
            assert abs(ss[i] - rs) < 1e-4 and abs(ms[i] - rm) < 1e-4, (size, i, ss[i], rs, ms[i], rm)
            assert abs(pp[i] - R.psnr(b, a)) < 1e-3
    same = torch.from_numpy(np.stack([pairs[0][1]])).cuda()
    s1, m1 = metrics.ssim_ms_ssim(same, same)
    assert abs(s1[0] - 1.0) < 1e-6 and abs(m1[0] - 1.0) < 1e-6
