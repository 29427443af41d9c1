"""ORACLE / TEST INFRASTRUCTURE: CPU twin of the device weight generator (see weights.c)."""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-C", _HERE], stdout=subprocess.DEVNULL)
        lib = C.CDLL(_SO)
        lib.oracle_fill_uniform.restype = None
        lib.oracle_fill_uniform.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_float, C.c_float]
        _lib = lib
    return _lib


def fill_uniform(n: int, seed: int, scale: float, offset: float) -> np.ndarray:
    """Uniform values in [offset - scale, offset + scale); identical to rdeic_fill_uniform."""
    out = np.empty(n, dtype=np.float32)
    _load().oracle_fill_uniform(out.ctypes.data, n, C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
                                float(np.float32(scale * 2.0 ** -23)), float(offset))
    return out
