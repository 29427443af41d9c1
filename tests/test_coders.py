"""Entropy coders: the C++ product coders (librdeic_hip.so, host code — runs without a GPU)
against the oracle restatement (oracle/coders_ref.py), the golden fixtures produced through
the reference's own compress/decompress call sites, and known-answer vectors."""
import os
import random

import numpy as np
import pytest
import torch

from oracle import coders_ref as cr
from rdeic_amd import coders

GOLD = os.path.join(os.path.dirname(__file__), "golden", "e2e_128.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.fixture(scope="module")
def tables():
    return coders.GaussianTables()


def test_scale_table_matches_reference(gold):
    assert np.array_equal(coders.get_scale_table().numpy(), gold["scale_table"])


def test_gaussian_tables_bitexact(gold, tables):
    """C++ pmf_to_quantized_cdf + table builder == restated compressai update() (fixture)."""
    ld = gold["quantized_cdf"].shape[1]
    assert tables.cdf_ld == ld
    assert np.array_equal(tables.cdf, gold["quantized_cdf"])
    assert np.array_equal(tables.cdf_length, gold["cdf_length"])
    assert np.array_equal(tables.offset, gold["offset"])
    # invariants: cdf[0]=0, cdf[len-1]=2^16, strictly increasing, 27,256 entries
    assert tables.levels == 64 and int(tables.cdf_length.max()) == 3133
    assert int(tables.cdf_length.sum()) == 27256
    for i in range(tables.levels):
        L = tables.cdf_length[i]
        row = tables.cdf[i, :L]
        assert row[0] == 0 and row[-1] == 65536 and np.all(np.diff(row) > 0)
        assert not tables.cdf[i, L:].any()  # zero tail past the row length


def test_pmf_to_quantized_cdf_random_vs_oracle():
    from rdeic_amd import _lib
    import ctypes as C
    rng = np.random.default_rng(0)
    for trial in range(50):
        n = int(rng.integers(2, 300))
        p = rng.random(n).astype(np.float32) ** 4
        p[rng.random(n) < 0.3] = 0.0
        if p.sum() == 0:
            p[0] = 1.0
        out = np.zeros(n + 1, dtype=np.uint32)
        _lib.call("rdeic_pmf_to_quantized_cdf", p.ctypes.data, n, 16, out.ctypes.data)
        ref = cr.pmf_to_quantized_cdf(p.tolist())
        assert out.tolist() == ref


def test_rans_golden_stream(gold, tables):
    """The reference's compress call site (with restated rANS) produced img*_y_string from
    (symbols, indexes); the C++ encoder must reproduce it byte for byte and decode it."""
    for i in range(2):
        sym, idx = gold[f"img{i}_symbols"], gold[f"img{i}_indexes"]
        data = coders.rans_encode(sym, idx, tables)
        assert data == gold[f"img{i}_y_string"].tobytes()
        dec = coders.RansDecoder(data)
        # decode in the reference's 20 per-stage chunks
        sizes = []
        for c in [8, 8, 8, 8, 16, 16, 32, 32, 64, 64]:
            sizes += [c * 8 * 4, c * 8 * 4]  # 128x128 image: y 8x8, squeezed 8x4
        assert sum(sizes) == sym.size
        pos, outs = 0, []
        for s in sizes:
            outs.append(dec.decode_stream(idx[pos:pos + s], tables))
            pos += s
        assert np.array_equal(np.concatenate(outs), sym)


def test_rans_roundtrip_escapes_and_oracle(tables):
    rng = np.random.default_rng(1)
    n = 4000
    idx = rng.integers(0, 64, n).astype(np.int32)
    # mostly in-range values plus large escapes (bypass chains), negative and positive
    sym = np.round(rng.normal(0, 1, n) * (tables.scale_table.numpy()[idx] + 0.1)).astype(np.int32)
    esc = rng.random(n) < 0.05
    sym[esc] = rng.integers(-100000, 100000, int(esc.sum()))
    data = coders.rans_encode(sym, idx, tables)
    ref_enc = cr.RansEncoderRef()
    ref_enc.encode_with_indexes(sym.tolist(), idx.tolist(), tables.cdf.tolist(), tables.cdf_length.tolist(),
                                tables.offset.tolist())
    assert data == ref_enc.flush()
    dec = coders.RansDecoder(data)
    assert np.array_equal(dec.decode_stream(idx, tables), sym)
    rdec = cr.RansDecoderRef()
    rdec.set_stream(data)
    assert rdec.decode_stream(idx.tolist(), tables.cdf.tolist(), tables.cdf_length.tolist(),
                              tables.offset.tolist()) == sym.tolist()


def test_rans_batch_equals_single(tables):
    rng = np.random.default_rng(2)
    count, n = 6, 3000
    idx = rng.integers(0, 64, (count, n)).astype(np.int32)
    sym = rng.integers(-3, 4, (count, n)).astype(np.int32)
    outs = coders.rans_encode_batch(sym, idx, tables, threads=4)
    for i in range(count):
        assert outs[i] == coders.rans_encode(sym[i], idx[i], tables)
    decs = [coders.RansDecoder(o) for o in outs]
    got = np.concatenate([coders.rans_decode_batch(decs, idx[:, :1000], tables, threads=3),
                          coders.rans_decode_batch(decs, idx[:, 1000:], tables, threads=3)], axis=1)
    assert np.array_equal(got, sym)


def test_rans_corrupt_stream_fails_cleanly(tables):
    from rdeic_amd._lib import BitstreamError
    rng = np.random.default_rng(3)
    idx = rng.integers(0, 64, 2000).astype(np.int32)
    sym = rng.integers(-20, 20, 2000).astype(np.int32)
    data = coders.rans_encode(sym, idx, tables)
    # truncation -> EBADMSG, never a crash or out-of-bounds read
    for cut in (0, 3, 8, len(data) // 2, len(data) - 4):
        dec = coders.RansDecoder(data[:cut])
        with pytest.raises(BitstreamError):
            dec.decode_stream(idx, tables)
    # random bit flips: must either decode (garbage) or raise BitstreamError
    for k in range(50):
        b = bytearray(data)
        pos = rng.integers(0, len(b))
        b[pos] ^= 1 << int(rng.integers(0, 8))
        dec = coders.RansDecoder(bytes(b))
        try:
            dec.decode_stream(idx, tables)
        except BitstreamError:
            pass


def test_torchac_uniform_kat():
    """Known answer: with 16384 codes every symbol costs exactly 14 bits, so the arithmetic code
    is the 14-bit MSB-first binary of each index, then the 2 termination bits '01', zero-padded:
    64 indices -> 898 bits -> 113 bytes."""
    rng = np.random.default_rng(4)
    for n in (64, 4, 1, 257):
        sym = rng.integers(0, 16384, n)
        data = coders.ac_encode_uniform(sym, 16384)
        bits = "".join(format(int(s), "014b") for s in sym) + "01"
        bits += "0" * ((-len(bits)) % 8)
        assert data == bytes(int(bits[k:k + 8], 2) for k in range(0, len(bits), 8))
        if n == 64:
            assert len(data) == 113
        assert np.array_equal(coders.ac_decode_uniform(data, n, 16384), sym.astype(np.int16))


def test_torchac_uniform_cdf_matches_restated_conversion():
    ref = cr.torchac_int_cdf(cr.uniform_cdf_float(16384)).numpy()
    assert np.array_equal(coders.uniform_cdf(16384), ref)


def test_torchac_nonuniform_vs_oracle():
    """The AC coder with a skewed CDF row (exercises E3 / pending bits) vs the restatement."""
    rng = np.random.default_rng(5)
    lp = 33
    p = rng.random(lp - 1) ** 3 + 1e-3
    cdf = np.concatenate([[0.0], np.cumsum(p / p.sum())]).astype(np.float32)
    cdf[-1] = 1.0
    row = cr.torchac_int_cdf(torch.from_numpy(cdf)).numpy()
    sym = rng.choice(lp - 1, size=3000, p=p / p.sum()).astype(np.int16)
    import ctypes as C
    from rdeic_amd import _lib
    out = np.empty(3000 * 4, dtype=np.uint8)
    n = C.c_size_t(0)
    _lib.call("rdeic_ac_encode", sym.ctypes.data, sym.size, row.ctypes.data, lp, out.ctypes.data, out.size,
              C.byref(n))
    data = out[:n.value].tobytes()
    assert data == cr.ac_encode(row.view(np.uint16), sym.tolist())
    dec = np.empty(3000, dtype=np.int16)
    _lib.call("rdeic_ac_decode", np.frombuffer(data, np.uint8).ctypes.data, len(data), 3000, row.ctypes.data, lp,
              dec.ctypes.data)
    assert np.array_equal(dec, sym)


def test_golden_z_string(gold):
    for i in range(2):
        idx = gold[f"img{i}_z_idx"].reshape(-1)
        assert coders.ac_encode_uniform(idx, 16384) == gold[f"img{i}_z_string"].tobytes()
        assert np.array_equal(coders.ac_decode_uniform(gold[f"img{i}_z_string"].tobytes(), idx.size, 16384), idx)


def test_tabled_encoder_bytes_and_reciprocals(tables, gold):
    """rdeic_rans_encode_batch_t (one reverse pass on precomputed reciprocal symbols) writes the
    same streams as the two-pass restatement of BufferedRansEncoder, escapes and multi-nibble
    bypass chains included, and every reciprocal division it uses is floor(x / freq) exactly,
    over the whole valid state range x < freq << 47 (sampled, plus both ends)."""
    import ctypes as C
    from rdeic_amd import _lib
    rng = np.random.default_rng(7)
    n = 20000
    idx = rng.integers(0, 64, size=(3, n)).astype(np.int32)
    sym = (rng.random((3, n)) < 0.2).astype(np.int32) * rng.integers(-60, 60, size=(3, n)).astype(np.int32)
    sym[0, :200] = rng.integers(-200000, 200000, size=200)
    sym[1, :20] = 2 ** 30
    sym[1, 20:40] = -2 ** 30
    assert coders.rans_encode_batch(sym, idx, tables, threads=3, tabled=True) == \
        coders.rans_encode_batch(sym, idx, tables, threads=3, tabled=False)
    # the golden file's y string (the reference's call order) from the tabled path
    y = coders.rans_encode_batch(gold["img0_symbols"][None], gold["img0_indexes"][None], tables)[0]
    assert y == gold["img0_y_string"].tobytes()
    lib, h, q = _lib.load(), tables.encoder_tables(), C.c_uint64()
    for row in range(0, 64, 3):
        L = int(tables.cdf_length[row])
        for v in sorted({0, 1, L // 2, L - 3, L - 2}):
            f = int(tables.cdf[row, v + 1] - tables.cdf[row, v])
            xs = [1, 2 ** 31, (f << 47) - 1] + [int(x) for x in rng.integers(1, f << 47, size=64, dtype=np.uint64)]
            for x in xs:
                assert lib.rdeic_rans_enc_quotient(h, row, v, x, C.byref(q)) == 0
                assert q.value == x // f, (row, v, f, x)


def test_default_threads_shared_among_local_ranks(monkeypatch):
    """The host coder pool divides the CPU quota among the node's ranks (one process per GPU under
    torch.distributed.run), so an 8-GPU node does not run 8 full-size pools per host."""
    monkeypatch.delenv("LOCAL_WORLD_SIZE", raising=False)
    n1 = coders.default_threads()
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    n4 = coders.default_threads()
    assert 1 <= n4 <= n1 <= 16
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1000")
    assert coders.default_threads() == 1


def test_default_threads_respects_per_rank_binding(monkeypatch):
    """The affinity set is divided among the node's ranks unless the ranks are bound to their own cores (declared
    by RDEIC_RANK_BOUND=1, or detected: an affinity set of at most 1 / LOCAL_WORLD_SIZE of the machine): a
    cpuset-limited container (affinity < os.cpu_count(), no quota) is shared by
    every rank, and RDEIC_CODER_THREADS overrides everything."""
    import os
    monkeypatch.delenv("RDEIC_CODER_THREADS", raising=False)
    monkeypatch.delenv("RDEIC_RANK_BOUND", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setattr(os, "cpu_count", lambda: 256)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(64)), raising=False)
    import builtins
    real_open = builtins.open

    def no_quota(path, *a, **k):
        if str(path) == "/sys/fs/cgroup/cpu.max":
            raise OSError("no cgroup")
        return real_open(path, *a, **k)
    monkeypatch.setattr(builtins, "open", no_quota)
    assert coders.default_threads() == 8          # cpuset of 64 shared by 8 ranks, not 8 x 16
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(6)), raising=False)
    assert coders.default_threads() == 6          # 6 x 8 ranks <= 256: a per-rank binding, detected
    monkeypatch.setattr(os, "cpu_count", lambda: 40)
    assert coders.default_threads() == 1          # 6 x 8 > 40: a shared cpuset, 6 // 8, at least one
    monkeypatch.setenv("RDEIC_RANK_BOUND", "1")
    assert coders.default_threads() == 6          # declared per-rank binding: 6 own cores
    monkeypatch.setenv("RDEIC_CODER_THREADS", "3")
    assert coders.default_threads() == 3
