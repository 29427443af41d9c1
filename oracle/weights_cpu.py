"""ORACLE / TEST INFRASTRUCTURE: CPU twin of the device weight generator (see weights.c)."""
import ctypes as C

import numpy as np

from ._clib import lib


def fill_uniform(n: int, seed: int, scale: float, offset: float) -> np.ndarray:
    """Uniform values in [offset - scale, offset + scale); identical to rdeic_fill_uniform."""
    out = np.empty(n, dtype=np.float32)
    lib().oracle_fill_uniform(out.ctypes.data, n, C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                              float(np.float32(scale * 2.0 ** -23)), float(offset))
    return out
