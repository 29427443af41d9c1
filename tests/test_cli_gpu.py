"""inference.py (the reference's CLI, reference inference.py:94-147) end to end on the GPU:
the written bitstream file equals the golden reference bytes and the PNG equals the golden
reconstruction (fp32 mode, within one uint8 level)."""
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "e2e_128.npz")


@pytest.mark.gpu
def test_cli_matches_golden(tmp_path):
    from PIL import Image
    import inference
    g = np.load(GOLDEN)
    src = tmp_path / "in"
    src.mkdir()
    Image.fromarray(g["img0_in"]).save(src / "kodim.png")
    inference.main(["--input", str(src), "--output", str(tmp_path / "out"), "--steps", "2", "--seed", "231",
                    "--sampler", "ddim"])
    data = (tmp_path / "out" / "data" / "kodim").read_bytes()
    assert data == g["img0_file"].tobytes()
    out = np.array(Image.open(tmp_path / "out" / "kodim.png"))
    assert np.abs(out.astype(int) - g["img0_image_out"][0].astype(int)).max() <= 1


@pytest.mark.gpu
def test_cli_default_ddpm_sampler(tmp_path):
    """The reference CLI's default sampler (--sampler ddpm): the bitstream is sampler-independent
    (golden bytes), the reconstruction comes from the spaced sampler (differs from the DDIM one)."""
    from PIL import Image
    import inference
    g = np.load(GOLDEN)
    src = tmp_path / "in"
    src.mkdir()
    Image.fromarray(g["img0_in"]).save(src / "kodim.png")
    inference.main(["--input", str(src), "--output", str(tmp_path / "out"), "--steps", "2", "--seed", "231"])
    assert (tmp_path / "out" / "data" / "kodim").read_bytes() == g["img0_file"].tobytes()
    out = np.array(Image.open(tmp_path / "out" / "kodim.png"))
    assert out.shape == g["img0_image_out"][0].shape
    assert np.abs(out.astype(int) - g["img0_image_out"][0].astype(int)).max() > 1


def test_pad_matches_reference_rule():
    import inference
    x = np.ones((100, 130, 3), np.uint8)
    y = inference.pad(x, 64)
    assert y.shape == (128, 192, 3) and y[:100, :130].all() and not y[100:].any() and not y[:, 130:].any()
    assert inference.pad(np.ones((64, 64, 3), np.uint8), 64).shape == (64, 64, 3)
