"""ORACLE / TEST INFRASTRUCTURE: loader for oracle/_build/liboracle.so (weights.c, rans.c)."""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        # Never build here: this can run inside a GPU test process after the device is up, and a
        # file push need not preserve mtimes. __graft_entry__.build() / `make -C oracle` build it.
        if not os.path.exists(_SO):
            raise ImportError(f"{_SO} is missing: run __graft_entry__.build() or `make -C oracle` first")
        L = C.CDLL(_SO)
        L.oracle_fill_uniform.restype = None
        L.oracle_fill_uniform.argtypes = [C.c_void_p, C.c_int64, C.c_uint64, C.c_float, C.c_float]
        P = C.c_void_p
        L.oracle_rans_encode.restype = C.c_int64
        L.oracle_rans_encode.argtypes = [P, P, C.c_int64, P, C.c_int64, P, P, P, C.c_int64]
        L.oracle_rans_dec_state_size.restype = C.c_int64
        L.oracle_rans_dec_init.restype = C.c_int
        L.oracle_rans_dec_init.argtypes = [P, P, C.c_int64]
        L.oracle_rans_decode.restype = C.c_int
        L.oracle_rans_decode.argtypes = [P, P, C.c_int64, P, C.c_int64, P, P, P]
        _lib = L
    return _lib
