"""The product model declares exactly the reference's parameters (names and shapes), so a
reference checkpoint loads unchanged and the synthetic weights line up with the golden run."""
import json
import os

import torch

from rdeic_amd import weights as W
from rdeic_amd.rdeic import RDEIC, make_schedule

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_param_names_and_shapes_match_reference():
    ref = json.load(open(os.path.join(GOLD, "param_shapes.json")))
    ref_params = {k: tuple(v) for k, v in ref.items() if W.is_param(k) and not k.endswith("scale_list")}
    # buffers of the reference that are not learnable parameters
    ref_params = {k: v for k, v in ref_params.items() if "gaussian_conditional" not in k}
    model = RDEIC(compute_dtype=torch.float32, device="cpu")
    mine = model.param_shapes()
    assert set(mine) == set(ref_params), (sorted(set(mine) - set(ref_params))[:5], sorted(set(ref_params) - set(mine))[:5])
    for k, v in ref_params.items():
        assert mine[k] == v, k
    n = sum(int(torch.tensor(s).prod()) for s in mine.values())
    assert 1.02e9 < n < 1.04e9  # ~1.03B parameters (UNet + control + VAE + compressor)


def test_schedule_matches_reference_buffers():
    import numpy as np
    g = np.load(os.path.join(GOLD, "e2e_128.npz"))
    s = make_schedule(1000, 0.00085, 0.0120)
    for k in ("betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_alphas_cumprod",
              "sqrt_one_minus_alphas_cumprod"):
        assert np.array_equal(s[k].numpy(), g["sched_" + k]), k
    # SURVEY §8a a10 values
    assert abs(float(s["sqrt_alphas_cumprod"][299]) - 0.76953435) < 1e-7
    assert abs(float(s["sqrt_one_minus_alphas_cumprod"][299]) - 0.63860542) < 1e-7


def test_ddim_timesteps():
    from rdeic_amd.ddim_sampler_relay import make_ddim_timesteps
    assert make_ddim_timesteps(2, 300).tolist() == [1, 151]
    assert make_ddim_timesteps(5, 300).tolist() == [1, 61, 121, 181, 241]


def test_rate_gain_calibration():
    """bench.py --bpp-sweep's rate knob: the calibration table is monotone and the interpolation
    returns its own points and stays between neighbours (rdeic_amd/weights.py)."""
    from rdeic_amd import weights as W
    pts = W.RATE_CALIBRATION_512
    assert all(a[0] < b[0] and a[1] < b[1] for a, b in zip(pts, pts[1:]))
    for g, b in pts:
        assert abs(W.rate_gain_for_bpp(b) - g) < 1e-4
    gains = [W.rate_gain_for_bpp(b) for b in (0.04, 0.08, 0.12)]
    assert 0.36 < gains[0] < 0.37 and 0.40 < gains[1] < 0.405 and 0.42 < gains[2] < 0.43
    assert W.rate_gain_for_bpp(0.001) == pts[0][0] and W.rate_gain_for_bpp(10.0) == pts[-1][0]
