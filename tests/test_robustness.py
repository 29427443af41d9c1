"""Robustness harness: the corruptors against the reference's own experiments/corruptors.py
(tests/golden/make_corruptor_golden.py -> corruptors.npz), and the HIP decode path under corrupted
bitstreams (never a crash; every failure is an exception the harness records; a failed decode leaves
the decoder and its launch plans intact)."""
import os
import struct

import numpy as np
import pytest
import torch

from rdeic_amd import robustness as R

GOLD = os.path.join(os.path.dirname(__file__), "golden", "corruptors.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def _cases(g, prefix):
    import re
    return sorted({k.split("_")[0] for k in g.files if re.match(prefix + r"\d+_", k)})


def test_byte_corruptors_match_reference(g):
    data = g["data"].tobytes()
    cases = _cases(g, "bytes")
    assert len(cases) == 8
    for c in cases:
        kind = g[c + "_kind"].tobytes().decode()
        cor = R.Corruptor("bitstream", kind, float(g[c + "_rate"]), int(g[c + "_seed"]))
        assert cor.corrupt_bytes(data) == g[c + "_out"].tobytes(), c


def test_latent_corruptors_match_reference(g):
    lat = torch.from_numpy(g["latent"])
    lo, hi = R.estimate_latent_range(lat)
    assert np.allclose([lo, hi], g["latent_range"], rtol=0, atol=0)
    for c in _cases(g, "lat"):
        mode = g[c + "_mode"].tobytes().decode()
        out = R.Corruptor("latent", mode, float(g[c + "_rate"]), int(g[c + "_seed"]), valid_range=(lo, hi)) \
            .corrupt_latent(lat)
        assert np.array_equal(out.numpy(), g[c + "_out"]), c


def test_corrupt_bitstream_file(tmp_path, g):
    src, dst = tmp_path / "a.bin", tmp_path / "b.bin"
    src.write_bytes(g["data"].tobytes())
    R.corrupt_bitstream_file(str(src), str(dst), "burst", float(g["bytes4_rate"]), int(g["bytes4_seed"]))
    assert dst.read_bytes() == g["bytes4_out"].tobytes()
    with pytest.raises(ValueError):
        R.Corruptor("bitstream", "additive", 0.1).corrupt_bytes(b"abc")


def test_header_corruption_is_an_exception():
    from rdeic_amd import bitstream
    body = bitstream.pack_body((8, 8), [[b"y" * 40], [b"z" * 9]])
    assert bitstream.unpack_body(body)[1] == (8, 8)
    with pytest.raises(ValueError):
        bitstream.unpack_body(body[:30])  # truncated y string
    with pytest.raises(struct.error):
        bitstream.unpack_body(body[:7])
    big = struct.pack(">3I", 8, 8, 5) + body[12:]  # n_strings corrupted
    with pytest.raises((ValueError, struct.error)):
        bitstream.unpack_body(big)


@pytest.mark.gpu
def test_corrupted_streams_fail_cleanly_and_decoder_recovers(gpu):
    """Decode many corrupted bodies (random + burst, header flips included): each either decodes or
    raises; afterwards a clean body still decodes bit-identically to before (plans and coders intact)."""
    from rdeic_amd import bitstream
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_image
    m = RDEIC().init_synthetic(rate_gain=0.4)
    img = torch.from_numpy(np.stack([synth_image(128, 128, 231 + i) for i in range(2)])).cuda()
    bodies = m.compress_images(img)
    lat0, hint0 = m.decompress_bodies([bodies[0]])
    lat0, hint0 = lat0.clone(), hint0.clone()
    n_fail = n_ok = 0
    for kind in ("random", "burst"):
        for rate in (0.001, 0.01, 0.05):
            for seed in range(3):
                r = R.try_decompress(m, R.Corruptor("bitstream", kind, rate, seed).corrupt_bytes(bodies[0]))
                if isinstance(r, Exception):
                    n_fail += 1
                else:
                    n_ok += 1
                    assert torch.isfinite(r[0]).all()
    # header flips: z shape and n_strings
    hdr = bytearray(bodies[0])
    hdr[0] ^= 0x80  # zh -> 2^31 + 2: implausible
    assert isinstance(R.try_decompress(m, bytes(hdr)), ValueError)
    assert n_fail + n_ok == 18
    lat1, hint1 = m.decompress_bodies([bodies[0]])
    assert torch.equal(lat0, lat1) and torch.equal(hint0, hint1)
    assert bitstream.unpack_body(bodies[1])[1] == bitstream.unpack_body(bodies[0])[1]


@pytest.mark.gpu
def test_bitstream_robustness_harness(gpu, tmp_path):
    from rdeic_amd.rdeic import RDEIC
    from rdeic_amd.synthetic import synth_image
    m = RDEIC().init_synthetic(rate_gain=0.4)
    img = torch.from_numpy(np.stack([synth_image(128, 128, 231 + i) for i in range(2)])).cuda()
    from rdeic_amd.synthetic import synth_context
    ctx = synth_context().cuda()
    recs = R.run_bitstream_robustness(m, img, ctx, "random", rates=[0.0, 0.02], seeds=[1, 2], steps=2)
    assert len(recs) == 2 * 2 * 2
    clean = [r for r in recs if r["error_rate"] == 0.0]
    assert all(not r["decode_failed"] and np.isfinite(r["psnr"]) and r["psnr"] > 0 for r in clean)
    for r in recs:
        assert r["decode_failed"] == (r["psnr"] == 0.0 and r.get("lpips") == 1.0) or not r["decode_failed"]
    R.write_csv(recs, str(tmp_path / "robustness.csv"))
    assert (tmp_path / "robustness.csv").read_text().count("\n") == len(recs) + 1
