"""The oracle (oracle/model_ref.py, CPU fp32 restatement) pinned against the golden fixtures
generated from the reference's own modules (tests/golden/make_golden.py): byte-identical
bitstreams, identical symbols/indexes and identical uint8 reconstructions."""
import numpy as np
import pytest
import torch

from oracle import coders_ref as cr
from oracle import model_ref as M
from oracle import rans_c

GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "e2e_128.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLDEN)


@pytest.fixture(scope="module")
def sd():
    return M.synthetic_state_dict()


@pytest.fixture(scope="module")
def tables():
    return M.Tables()


def test_tables_match_golden(g, tables):
    assert np.array_equal(np.asarray(tables.cdf), g["quantized_cdf"])
    assert np.array_equal(np.asarray(tables.lens), g["cdf_length"])
    assert np.array_equal(np.asarray(tables.off), g["offset"])


@pytest.mark.parametrize("i", [0, 1])
def test_oracle_compress_matches_golden(g, sd, tables, i):
    x = torch.tensor(np.stack([g[f"img{i}_in"]]) / 255.0, dtype=torch.float32).permute(0, 3, 1, 2).contiguous()
    c = M.vae_encode_hc(sd, x * 2 - 1)
    np.testing.assert_allclose(c.numpy(), g[f"img{i}_vae_c"], atol=1e-4)
    body, sym, idx = M.compress(sd, c * 0.18215, tables, coder="py")
    assert np.array_equal(sym, g[f"img{i}_symbols"]) and np.array_equal(idx, g[f"img{i}_indexes"])
    assert body == g[f"img{i}_file"].tobytes()
    body_c, _, _ = M.compress(sd, c * 0.18215, tables, coder="c")
    assert body_c == body
    cl, hint = M.decompress(sd, body, tables, coder="c")
    np.testing.assert_allclose(cl.numpy(), g[f"img{i}_c_latent"], atol=1e-5)
    np.testing.assert_allclose(hint.numpy(), g[f"img{i}_guide_hint"], atol=1e-5)


def test_oracle_end_to_end(g, sd, tables):
    out, body = M.codec_image(sd, tables, g["img0_in"], torch.from_numpy(g["context"]),
                              torch.from_numpy(g["img0_noise"]), steps=2, coder="c")
    assert body == g["img0_file"].tobytes()
    assert np.abs(out.astype(int) - g["img0_image_out"][0].astype(int)).max() <= 1


def test_rans_c_twin_matches_python():
    rng = np.random.default_rng(5)
    st = cr.get_scale_table()
    cdf, lens, off = cr.gaussian_tables(st)
    n = 3000
    idx = rng.integers(0, 64, n).astype(np.int32)
    sym = np.round(rng.normal(0, 1, n) * (idx + 1) * 0.8).astype(np.int32)
    sym[::97] = 40000  # bypass-coded outliers
    sym[5::101] = -40000
    e = cr.RansEncoderRef()
    e.encode_with_indexes(sym.tolist(), idx.tolist(), cdf.tolist(), lens.tolist(), off.tolist())
    ref = e.flush()
    ec = rans_c.RansEncoderC()
    ec.encode_with_indexes(sym, idx, cdf, lens, off)
    assert ec.flush() == ref
    d = rans_c.RansDecoderC()
    d.set_stream(ref)
    half = n // 2
    out = np.concatenate([d.decode_stream(idx[:half], cdf, lens, off), d.decode_stream(idx[half:], cdf, lens, off)])
    assert np.array_equal(out, sym)
