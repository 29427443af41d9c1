"""ctypes binding of librdeic_hip.so (the C ABI declared in include/rdeic_hip.h).

The library is the product: there is no Python / torch fallback for any kernel. Loading
fails loudly when the shared object is missing, and every call raises on a non-zero
status code.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RDEIC_LIB") or os.path.join(_HERE, "lib", "librdeic_hip.so")

EINVAL, ENOSPC, EBADMSG, ELAUNCH = -22, -28, -74, -5
_ERRNAMES = {EINVAL: "EINVAL (bad argument/shape)", ENOSPC: "ENOSPC (output capacity)",
             EBADMSG: "EBADMSG (corrupt or truncated bitstream)", ELAUNCH: "kernel launch failure"}


class RdeicError(RuntimeError):
    def __init__(self, fn: str, code: int):
        super().__init__(f"{fn} failed: {code} {_ERRNAMES.get(code, '')}")
        self.code = code


class BitstreamError(RdeicError, ValueError):
    """Corrupt / truncated bitstream (the reference's 'decode failure')."""


class ConvDesc(C.Structure):
    """Mirror of rdeic_conv_desc."""
    _fields_ = [
        ("in0", C.c_void_p), ("in1", C.c_void_p),
        ("c0", C.c_int32), ("c1", C.c_int32), ("ld0", C.c_int32), ("ld1", C.c_int32),
        ("n", C.c_int32), ("h", C.c_int32), ("w", C.c_int32), ("up2", C.c_int32),
        ("weight", C.c_void_p), ("wld", C.c_int32),
        ("bias", C.c_void_p),
        ("cout", C.c_int32), ("kh", C.c_int32), ("kw", C.c_int32), ("stride", C.c_int32),
        ("pad_t", C.c_int32), ("pad_l", C.c_int32),
        ("ho", C.c_int32), ("wo", C.c_int32),
        ("gn_ab", C.c_void_p), ("gn_silu", C.c_int32),
        ("emb", C.c_void_p), ("emb_ld", C.c_int32),
        ("act", C.c_int32), ("act_param", C.c_float),
        ("res", C.c_void_p), ("res_ld", C.c_int32),
        ("out", C.c_void_p), ("out_ld", C.c_int32), ("out_mode", C.c_int32),
        ("dtype", C.c_int32), ("out_f32", C.c_int32),
        ("batch", C.c_int32), ("in_bs", C.c_int64), ("w_bs", C.c_int64), ("out_bs", C.c_int64),
        ("gn_part", C.c_void_p), ("gn_hw", C.c_int32), ("reserved", C.c_int32),
        ("ln_rows", C.c_void_p), ("ln_colsum", C.c_void_p),
    ]


class GemmDesc(C.Structure):
    """Mirror of rdeic_gemm_desc (strided batched GEMM, train.hip)."""
    _fields_ = [
        ("a", C.c_void_p), ("a_bs1", C.c_int64), ("a_bs2", C.c_int64), ("a_sm", C.c_int64), ("a_sk", C.c_int64),
        ("b", C.c_void_p), ("b_bs1", C.c_int64), ("b_bs2", C.c_int64), ("b_sk", C.c_int64), ("b_sn", C.c_int64),
        ("c", C.c_void_p), ("c_bs1", C.c_int64), ("c_bs2", C.c_int64), ("c_sm", C.c_int64),
        ("batch", C.c_int32), ("nb2", C.c_int32), ("m", C.c_int32), ("n", C.c_int32), ("k", C.c_int32),
        ("ksplit", C.c_int32), ("dtype", C.c_int32), ("c_f32", C.c_int32),
        ("alpha", C.c_float), ("beta", C.c_float), ("rsum", C.c_void_p), ("rsum_bs", C.c_int64),
    ]


_p, _i32, _i64, _u64, _f, _sz = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_size_t

# name -> (restype, argtypes). Every symbol of include/rdeic_hip.h appears here.
PROTOTYPES = {
    "rdeic_version": (C.c_int, []),
    "rdeic_abi_count": (C.c_int, []),
    "rdeic_conv2d": (C.c_int, [C.POINTER(ConvDesc), _p]),
    "rdeic_conv2d_splitk": (C.c_int, [C.POINTER(ConvDesc), _i32, _p, C.c_size_t, _p]),
    "rdeic_conv2d_tile": (C.c_int, [C.POINTER(ConvDesc), _i32, _p]),
    "rdeic_prof_start": (C.c_int, [_i32, _i32]),
    "rdeic_prof_stop": (C.c_int, []),
    "rdeic_launch_count": (C.c_int64, [_i32]),
    "rdeic_launch_count_reset": (C.c_int, []),
    "rdeic_layernorm_rowstats": (C.c_int, [C.c_void_p, _i32, _i32, _i32, C.c_float, C.c_void_p, C.c_void_p]),
    "rdeic_prof_read": (C.c_int, [_i32, C.POINTER(C.c_int64), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "rdeic_prof_read_keys": (C.c_int, [_i32, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_double),
                                       C.POINTER(C.c_double), _i32]),
    "rdeic_groupnorm_ws_floats": (_sz, [_i32, _i32, _i32]),
    "rdeic_groupnorm_stats": (C.c_int, [_p, _i32, _i32, _p, _i32, _i32, _i32, _i32, _i32, _f, _p, _p, _p, _p,
                                        _i32, _p]),
    "rdeic_groupnorm_apply": (C.c_int, [_p, _i32, _i32, _i32, _i32, _p, _i32, _i32, _f, _p, _i32, _i32, _p]),
    "rdeic_set_conv_path": (C.c_int, [_i32]),
    "rdeic_set_conv_option": (C.c_int, [_i32, _i32]),
    "rdeic_layernorm": (C.c_int, [_p, _i32, _i32, _i32, _p, _p, _f, _p, _i32, _i32, _p]),
    "rdeic_softmax_rows": (C.c_int, [_p, _i64, _i32, _f, _p, _i32, _p]),
    "rdeic_transpose": (C.c_int, [_p, _i32, _i32, _i32, _p, _i32, _i32, _i64, _i64, _i32, _p]),
    "rdeic_attention": (C.c_int, [_p, _i32, _p, _i32, _p, _i32, _p, _i32, _i32, _i32, _i32, _i32, _i32, _f,
                                  _i32, _i32, _p]),
    "rdeic_geglu": (C.c_int, [_p, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_nchw_to_nhwc": (C.c_int, [_p, _i32, _i32, _i32, _i32, _f, _f, _p, _i32, _i32, _p]),
    "rdeic_nhwc_to_nchw": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _f, _f, _p, _i32, _p]),
    "rdeic_axpby": (C.c_int, [_p, _p, _i32, _i32, _p, _p, _p, _p]),
    "rdeic_timestep_embedding": (C.c_int, [_p, _p, _i32, _i32, _p, _p]),
    "rdeic_ddim_step": (C.c_int, [_p, _p, _i64, _f, _f, _f, _f, _p, _p, _p]),
    "rdeic_spaced_step": (C.c_int, [_p, _p, _p, _i64, _f, _f, _f, _f, _f, _p, _p, _p]),
    "rdeic_cfg_combine": (C.c_int, [_p, _p, _i64, _f, _p, _p]),
    "rdeic_silu_f32": (C.c_int, [_p, _p, _i64, _p]),
    "rdeic_image_u8_to_nhwc": (C.c_int, [_p, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_nhwc_to_image_u8": (C.c_int, [_p, _i32, _i32, _i32, _i32, _p, _i32, _p]),
    "rdeic_image_mse": (C.c_int, [_p, _p, _i32, _i64, _p, _p]),
    "rdeic_fill_uniform": (C.c_int, [_p, _i64, _u64, _f, _f, _p]),
    "rdeic_pack_conv_weight": (C.c_int, [_p, _i32, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_cast": (C.c_int, [_p, _i32, _p, _i32, _i64, _p]),
    "rdeic_ckbd_encode": (C.c_int, [_p, _i32, _p, _i32, _i32, _i32, _i32, _i32, _i32, _p, _i32, _f, _p, _p,
                                    _i64, _i64, _p, _i32, _p, _i32, _i32, _p]),
    "rdeic_ckbd_indexes": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _i32, _p, _i32, _f, _p, _i64, _i64,
                                     _i32, _p]),
    "rdeic_ckbd_dequant": (C.c_int, [_p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _p, _i32, _p,
                                     _i32, _i32, _p]),
    "rdeic_vq_argmin": (C.c_int, [_p, _p, _p, _i32, _i32, _p, _p]),
    "rdeic_gather_rows": (C.c_int, [_p, _i32, _p, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_row_sqnorm": (C.c_int, [_p, _i32, _i32, _i32, _p, _i32, _p]),
    "rdeic_pmf_to_quantized_cdf": (C.c_int, [_p, _i32, _i32, _p]),
    "rdeic_build_gaussian_tables": (C.c_int, [_p, _p, _i32, _i32, _p, _i32, _p, _p]),
    "rdeic_rans_encode": (C.c_int, [_p, _p, _sz, _p, _i32, _p, _p, _i32, _p, _sz, C.POINTER(_sz)]),
    "rdeic_rans_encode_batch": (C.c_int, [_i32, _p, _p, _sz, _sz, _p, _i32, _p, _p, _i32, _p, _sz, _p, _i32]),
    "rdeic_image_ssim_ws_floats": (C.c_size_t, [_i32, _i32, _i32, _i32]),
    "rdeic_image_ssim": (C.c_int, [_p, _p, _i32, _i32, _i32, _i32, _p, C.c_size_t, _p, _p]),
    "rdeic_groupnorm_parts_floats": (C.c_size_t, [_i64, _i32, _i32]),
    "rdeic_groupnorm_parts_ab": (C.c_int, [_p, _i32, _p, _i32, _i32, _i32, _i32, _f, _p, _p, _p, _p]),
    "rdeic_groupnorm_parts_apply": (C.c_int, [_p, _i32, _p, _i32, _p, _i32, _p, _i32, _i32, _i32, _i32, _f, _p, _p,
                                              _i32, _p, _p, _i32, _p]),
    "rdeic_rans_enc_tables_create": (_p, [_p, _i32, _p, _p, _i32]),
    "rdeic_rans_enc_tables_destroy": (None, [_p]),
    "rdeic_rans_encode_batch_t": (C.c_int, [_p, _i32, _p, _p, _sz, _sz, _p, _sz, _p, _i32]),
    "rdeic_rans_enc_quotient": (C.c_int, [_p, _i32, _i32, C.c_uint64, C.POINTER(C.c_uint64)]),
    "rdeic_rans_dec_open": (_p, [_p, _sz]),
    "rdeic_rans_decode": (C.c_int, [_p, _p, _sz, _p, _i32, _p, _p, _i32, _p]),
    "rdeic_rans_decode_batch": (C.c_int, [_i32, _p, _p, _sz, _sz, _p, _i32, _p, _p, _i32, _p, _i32]),
    "rdeic_rans_dec_close": (None, [_p]),
    "rdeic_ac_encode": (C.c_int, [_p, _sz, _p, _i32, _p, _sz, C.POINTER(_sz)]),
    "rdeic_ac_decode": (C.c_int, [_p, _sz, _sz, _p, _i32, _p]),
    "rdeic_ac_uniform_cdf": (C.c_int, [_i32, _p]),
    # adapter fine-tune step (train.hip)
    "rdeic_gemm_strided": (C.c_int, [C.POINTER(GemmDesc), _p]),
    "rdeic_pack_conv_weight_dgrad": (C.c_int, [_p, _i32, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_pack_batch": (C.c_int, [_p, _i32, _i64, _i32, _i32, _p]),
    "rdeic_zero_insert2": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_sum_pool2": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_pixel_unshuffle2": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_im2col": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _p,
                               _i64, _i32, _p]),
    "rdeic_wgrad_finalize": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _p, _p, _p]),
    "rdeic_col_sum_ws_floats": (_sz, [_i64, _i32, _i32]),
    "rdeic_col_sum": (C.c_int, [_p, _i64, _i32, _i32, _i32, _p, _i32, _p, _sz, _i32, _p]),
    "rdeic_act_fwd": (C.c_int, [_p, _i64, _i32, _i32, _p, _i32, _i32, _f, _p, _i32, _i32, _p]),
    "rdeic_act_bwd": (C.c_int, [_p, _i32, _p, _i32, _i64, _i32, _i32, _f, _p, _i32, _i32, _p]),
    "rdeic_gn_train_ws_doubles": (_sz, [_i32, _i32, _i32]),
    "rdeic_gn_train_fwd": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _f, _p, _p, _p, _p, _p, _i32, _p]),
    "rdeic_gn_train_bwd": (C.c_int, [_p, _i32, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _i32, _p, _i32, _p, _p,
                                     _i32, _p, _p, _i32, _p]),
    "rdeic_gn_train_bwd_res": (C.c_int, [_p, _i32, _p, _i32, _i32, _i32, _i32, _i32, _p, _p, _p, _i32, _p, _i32, _p,
                                         _i32, _p, _p, _i32, _p, _p, _i32, _p]),
    "rdeic_layernorm_bwd_ws_floats": (_sz, [_i64, _i32]),
    "rdeic_layernorm_bwd": (C.c_int, [_p, _i32, _i64, _i32, _p, _f, _p, _i32, _p, _i32, _p, _p, _i32, _p, _sz, _i32,
                                      _p]),
    "rdeic_layernorm_bwd_res": (C.c_int, [_p, _i32, _i64, _i32, _p, _f, _p, _i32, _p, _i32, _p, _i32, _p, _p, _i32, _p,
                                          _sz, _i32, _p]),
    "rdeic_softmax_bwd_rows": (C.c_int, [_p, _p, _i64, _i32, _f, _p, _i32, _p]),
    "rdeic_geglu_bwd": (C.c_int, [_p, _i32, _i64, _i32, _p, _i32, _p, _i32, _i32, _p]),
    "rdeic_ckbd_train_anchor": (C.c_int, [_p, _i32, _p, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_ckbd_mask": (C.c_int, [_p, _i32, _i32, _i32, _i32, _i32, _i32, _p, _i32, _i32, _p]),
    "rdeic_ckbd_train_ws_doubles": (_sz, [_i32, _i32, _i32, _i32]),
    "rdeic_ckbd_train_lik": (C.c_int, [_p, _i32, _p, _i32, _p, _i32, _p, _i32, _i32, _i32, _i32, _p, _i32, _p, _p,
                                       _i32, _p]),
    "rdeic_ckbd_train_lik_bwd": (C.c_int, [_p, _i32, _p, _i32, _p, _i32, _p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p,
                                           _i32, _p, _i32, _p, _i32, _i32, _p]),
    "rdeic_vq_train": (C.c_int, [_p, _p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _f, _f, _f, _p, _p, _p, _p]),
    "rdeic_vq_z_grad": (C.c_int, [_p, _p, _p, _i64, _p, _f, _p, _i32, _p]),
    "rdeic_scale_dev": (C.c_int, [_p, _i64, _p, _p, _i32, _p]),
    "rdeic_adamw": (C.c_int, [_p, _p, _p, _p, _i64, _f, _f, _f, _f, _f, _i32, _p]),
    "rdeic_adamw_dev": (C.c_int, [_p, _p, _p, _p, _i64, _f, _f, _f, _f, _f, _p, _p]),
}

_lib = None
_lock = threading.Lock()


def load() -> C.CDLL:
    """Load librdeic_hip.so once. Raises if it has not been built (no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"librdeic_hip.so not built at {LIB_PATH}; run `make` (or __graft_entry__.build()).")
        # torch must own the HIP runtime first so this library binds to the same libamdhip64 instance
        import torch  # noqa: F401
        lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(lib, name)  # AttributeError here = a declared export is missing
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(name: str, rc: int) -> None:
    if rc != 0:
        if rc == EBADMSG:
            raise BitstreamError(name, rc)
        raise RdeicError(name, rc)


# When set to a list, every call() is also appended as (name, fn, args, tag) — rdeic_amd/plan.py
# records a fixed-shape region's launch sequence this way and replays it without the Python layer
# logic. `tag` = (kind, work, meta) marks launches bench.py times with events ("conv", FLOPs, ...).
RECORDER = None


def call(name: str, *args, tag=None) -> None:
    fn = getattr(load(), name)
    if RECORDER is not None:
        RECORDER.append((name, fn, args, tag))
    rc = fn(*args)
    check(name, rc)
