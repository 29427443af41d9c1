"""ORACLE / TEST INFRASTRUCTURE: ctypes front of oracle/rans.c with the same interface as
coders_ref.RansEncoderRef / RansDecoderRef (used for the CPU baseline at full image sizes)."""
import ctypes as C
from typing import List

import numpy as np

from ._clib import lib


class _Tables:
    def __init__(self, cdfs, cdf_sizes, offsets):
        self.cdf = np.ascontiguousarray(np.asarray(cdfs, dtype=np.int32))
        self.lens = np.ascontiguousarray(np.asarray(cdf_sizes, dtype=np.int32))
        self.offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.int32))


def _tables(cdfs, cdf_sizes, offsets):
    if isinstance(cdfs, _Tables):
        return cdfs
    return _Tables(cdfs, cdf_sizes, offsets)


class RansEncoderC:
    def __init__(self):
        self._sym, self._idx, self._t = [], [], None

    def encode_with_indexes(self, symbols, indexes, cdfs, cdf_sizes, offsets):
        self._t = _tables(cdfs, cdf_sizes, offsets)
        self._sym.append(np.asarray(symbols, dtype=np.int32).reshape(-1))
        self._idx.append(np.asarray(indexes, dtype=np.int32).reshape(-1))

    def flush(self) -> bytes:
        sym = np.ascontiguousarray(np.concatenate(self._sym)) if self._sym else np.zeros(0, np.int32)
        idx = np.ascontiguousarray(np.concatenate(self._idx)) if self._idx else np.zeros(0, np.int32)
        cap = 64 * sym.size + 64
        out = np.empty(cap, dtype=np.uint8)
        t = self._t or _Tables(np.zeros((1, 2), np.int32), [2], [0])
        n = lib().oracle_rans_encode(sym.ctypes.data, idx.ctypes.data, sym.size, t.cdf.ctypes.data,
                                     t.cdf.shape[1], t.lens.ctypes.data, t.offs.ctypes.data,
                                     out.ctypes.data, cap)
        if n < 0:
            raise RuntimeError("oracle rANS encode failed")
        self._sym, self._idx = [], []
        return out[:n].tobytes()


class RansDecoderC:
    def set_stream(self, data: bytes):
        self._buf = np.frombuffer(bytes(data), dtype=np.uint8).copy()
        self._st = C.create_string_buffer(int(lib().oracle_rans_dec_state_size()))
        if lib().oracle_rans_dec_init(self._st, self._buf.ctypes.data, self._buf.size):
            raise ValueError("truncated rANS stream")

    def decode_stream(self, indexes, cdfs, cdf_sizes, offsets) -> List[int]:
        t = _tables(cdfs, cdf_sizes, offsets)
        idx = np.ascontiguousarray(np.asarray(indexes, dtype=np.int32).reshape(-1))
        out = np.empty(idx.size, dtype=np.int32)
        if lib().oracle_rans_decode(self._st, idx.ctypes.data, idx.size, t.cdf.ctypes.data, t.cdf.shape[1],
                                    t.lens.ctypes.data, t.offs.ctypes.data, out.ctypes.data):
            raise ValueError("rANS stream exhausted")
        return out
