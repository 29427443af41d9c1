"""Host entropy coders (C++ in librdeic_hip.so) behind the reference's coder call sites.

* GaussianTables   — compressai GaussianConditional.update() (model/compression.py:275-280):
  the float32 pmf is computed exactly as compressai does it (torch CPU erfc at model load, like
  the reference, which runs update() on CPU before .to(device)); quantisation to 16-bit CDFs
  (pmf_to_quantized_cdf) runs in C++.
* RansEncoder / rans_encode_batch — BufferedRansEncoder.encode_with_indexes + flush
  (compression.py:166,205-206), one independent stream per image, encoded on host threads.
* RansDecoder      — RansDecoder.set_stream / decode_stream (compression.py:230-231,
  utils/ckbd.py:103,112); the stream state persists across the 20 per-stage calls.
* ac_encode_uniform / ac_decode_uniform — torchac.encode_float_cdf / decode_float_cdf for the
  uniform hyper-latent CDF (utils/ckbd.py:130-141).
"""
from __future__ import annotations

import ctypes as C
import math
import os
from typing import List, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import call

TAIL_MASS = 1e-9
SCALE_BOUND = 0.11


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def get_scale_table(min_=0.11, max_=256.0, levels=64) -> torch.Tensor:
    """utils/func.py:10-13."""
    return torch.exp(torch.linspace(math.log(min_), math.log(max_), levels))


class GaussianTables:
    """quantized_cdf [levels][ld] int32, cdf_length [levels], offset [levels] + the scale table."""

    def __init__(self, scale_table: torch.Tensor = None):
        if scale_table is None:
            scale_table = get_scale_table()
        self.scale_table = scale_table.detach().float().cpu().contiguous()
        st = self.scale_table
        import scipy.stats
        multiplier = -float(scipy.stats.norm.ppf(TAIL_MASS / 2))
        pmf_center = torch.ceil(st * multiplier).int()
        pmf_length = 2 * pmf_center + 1
        max_length = int(pmf_length.max().item())
        samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
        scale = st.unsqueeze(1).float()
        half, const = float(0.5), float(-(2 ** -0.5))
        upper = half * torch.erfc(const * ((0.5 - samples) / scale))
        lower = half * torch.erfc(const * ((-0.5 - samples) / scale))
        pmf = upper - lower
        tail = 2 * lower[:, :1]
        levels = st.numel()
        rows = np.zeros((levels, max_length + 1), dtype=np.float32)
        lens = pmf_length.numpy().astype(np.int32)
        for i in range(levels):
            rows[i, :lens[i]] = pmf[i, :lens[i]].numpy()
            rows[i, lens[i]] = tail[i, 0].item()
        self.levels = levels
        self.cdf_ld = max_length + 2
        self.cdf = np.zeros((levels, self.cdf_ld), dtype=np.int32)
        self.cdf_length = np.zeros(levels, dtype=np.int32)
        call("rdeic_build_gaussian_tables", _np_ptr(rows), _np_ptr(lens), levels, rows.shape[1], _np_ptr(self.cdf),
             self.cdf_ld, _np_ptr(self.cdf_length), None)
        self.offset = (-pmf_center).numpy().astype(np.int32)
        self._dev = None
        self._enc = None

    def encoder_tables(self) -> int:
        """Handle of the precomputed encoder symbols (rdeic_rans_enc_tables_create), built once."""
        if self._enc is None:
            lib = _lib.load()
            h = lib.rdeic_rans_enc_tables_create(_np_ptr(self.cdf), self.cdf_ld, _np_ptr(self.cdf_length),
                                                 _np_ptr(self.offset), self.levels)
            if not h:
                raise ValueError("rdeic_rans_enc_tables_create rejected the CDF tables")
            self._enc = h
        return self._enc

    def __del__(self):
        try:
            if self._enc:
                _lib.load().rdeic_rans_enc_tables_destroy(self._enc)
                self._enc = None
        except Exception:
            pass

    def device_scale_table(self, device) -> torch.Tensor:
        if self._dev is None or self._dev.device != torch.device(device):
            self._dev = self.scale_table.to(device)
        return self._dev


def default_threads() -> int:
    """Host coder threads per call, at most 16. RDEIC_CODER_THREADS overrides. Otherwise: the CPUs
    this process may run on (affinity set), capped by the cgroup CPU quota (a GPU box shows 256 CPUs
    but grants 16). The quota is shared by every rank of this node (LOCAL_WORLD_SIZE, one process
    per GPU), so each rank takes quota / LWS. The affinity set is divided the same way unless the
    launcher says it bound each rank to its own cores (RDEIC_RANK_BOUND=1): a cpuset-limited container
    also shows fewer CPUs than os.cpu_count(), and its ranks share that set."""
    env = os.environ.get("RDEIC_CODER_THREADS")
    if env:
        return max(1, int(env))
    try:
        lws = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    except ValueError:
        lws = 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    # ranks bound to their own cores: declared (RDEIC_RANK_BOUND=1), or an affinity set no larger than this rank's
    # share of the machine (a launcher's per-rank binding, e.g. 6 cores of 48 with 8 ranks)
    bound = os.environ.get("RDEIC_RANK_BOUND") == "1" or (lws > 1 and aff * lws <= (os.cpu_count() or aff))
    n = aff if bound else aff // lws
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period) // lws))
    except (OSError, ValueError):
        pass
    return max(1, min(16, n))


def rans_encode(symbols: np.ndarray, indexes: np.ndarray, t: GaussianTables) -> bytes:
    sym = np.ascontiguousarray(symbols, dtype=np.int32)
    idx = np.ascontiguousarray(indexes, dtype=np.int32)
    cap = 4 * (sym.size * 4 + 16)
    out = np.empty(cap, dtype=np.uint8)
    n = C.c_size_t(0)
    call("rdeic_rans_encode", _np_ptr(sym), _np_ptr(idx), sym.size, _np_ptr(t.cdf), t.cdf_ld, _np_ptr(t.cdf_length),
         _np_ptr(t.offset), t.levels, _np_ptr(out), cap, C.byref(n))
    return out[:n.value].tobytes()


def rans_encode_batch(symbols: np.ndarray, indexes: np.ndarray, t: GaussianTables, threads: int = None,
                      tabled: bool = True) -> List[bytes]:
    """symbols / indexes [count, n] int32 -> one rANS stream per row (threads across rows).
    tabled (default): one reverse pass on the precomputed encoder symbols (no divisions);
    tabled=False: the two-pass restatement (BufferedRansEncoder's symbol list, then flush)."""
    sym = np.ascontiguousarray(symbols, dtype=np.int32)
    idx = np.ascontiguousarray(indexes, dtype=np.int32)
    count, n = sym.shape
    cap = 4 * (n * 4 + 16)
    out = np.empty((count, cap), dtype=np.uint8)
    lens = np.zeros(count, dtype=np.uint64)
    if tabled:
        call("rdeic_rans_encode_batch_t", t.encoder_tables(), count, _np_ptr(sym), _np_ptr(idx), n, n, _np_ptr(out),
             cap, _np_ptr(lens), threads or default_threads())
    else:
        call("rdeic_rans_encode_batch", count, _np_ptr(sym), _np_ptr(idx), n, n, _np_ptr(t.cdf), t.cdf_ld,
             _np_ptr(t.cdf_length), _np_ptr(t.offset), t.levels, _np_ptr(out), cap, _np_ptr(lens),
             threads or default_threads())
    return [out[i, :int(lens[i])].tobytes() for i in range(count)]


class RansDecoder:
    """One bitstream; decode_stream may be called repeatedly (state persists)."""

    def __init__(self, data: bytes):
        self._buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        lib = _lib.load()
        self.handle = lib.rdeic_rans_dec_open(_np_ptr(self._buf) if self._buf.size else None, self._buf.size)
        if not self.handle:
            raise MemoryError("rdeic_rans_dec_open failed")

    def decode_stream(self, indexes: np.ndarray, t: GaussianTables) -> np.ndarray:
        idx = np.ascontiguousarray(indexes, dtype=np.int32)
        out = np.empty(idx.size, dtype=np.int32)
        call("rdeic_rans_decode", self.handle, _np_ptr(idx), idx.size, _np_ptr(t.cdf), t.cdf_ld,
             _np_ptr(t.cdf_length), _np_ptr(t.offset), t.levels, _np_ptr(out))
        return out

    def close(self):
        if self.handle:
            _lib.load().rdeic_rans_dec_close(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def rans_decode_batch(decoders: Sequence[RansDecoder], indexes: np.ndarray, t: GaussianTables,
                      out: np.ndarray = None, threads: int = None) -> np.ndarray:
    """indexes [count, n] -> symbols [count, n]; decoder i consumes row i."""
    idx = np.ascontiguousarray(indexes, dtype=np.int32)
    count, n = idx.shape
    if out is None:
        out = np.empty((count, n), dtype=np.int32)
    handles = (C.c_void_p * count)(*[d.handle for d in decoders])
    call("rdeic_rans_decode_batch", count, C.cast(handles, C.c_void_p), _np_ptr(idx), n, n, _np_ptr(t.cdf), t.cdf_ld,
         _np_ptr(t.cdf_length), _np_ptr(t.offset), t.levels, _np_ptr(out), threads or default_threads())
    return out


_UNIFORM = {}


def uniform_cdf(codebook_size: int) -> np.ndarray:
    if codebook_size not in _UNIFORM:
        row = np.empty(codebook_size + 1, dtype=np.int16)
        call("rdeic_ac_uniform_cdf", codebook_size, _np_ptr(row))
        _UNIFORM[codebook_size] = row
    return _UNIFORM[codebook_size]


def ac_encode_uniform(indices: np.ndarray, codebook_size: int) -> bytes:
    """compress_hyper_latent (utils/ckbd.py:130-134): indices cast to int16, uniform CDF."""
    sym = np.ascontiguousarray(np.asarray(indices).reshape(-1), dtype=np.int16)
    if sym.size and (sym.min() < 0 or sym.max() >= codebook_size):
        raise ValueError(f"sym.max() == {sym.max()}, should be <= Lp - 1")
    row = uniform_cdf(codebook_size)
    cap = sym.size * 4 + 16
    out = np.empty(cap, dtype=np.uint8)
    n = C.c_size_t(0)
    call("rdeic_ac_encode", _np_ptr(sym) if sym.size else None, sym.size, _np_ptr(row), row.size, _np_ptr(out), cap,
         C.byref(n))
    return out[:n.value].tobytes()


def ac_decode_uniform(data: bytes, count: int, codebook_size: int) -> np.ndarray:
    """decompress_hyper_latent (utils/ckbd.py:137-141) -> int16 [count]."""
    buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
    row = uniform_cdf(codebook_size)
    out = np.empty(count, dtype=np.int16)
    call("rdeic_ac_decode", _np_ptr(buf) if buf.size else None, buf.size, count, _np_ptr(row), row.size,
         _np_ptr(out))
    return out
