"""Tensor-level wrappers over the C ABI (device buffers are torch tensors; torch is plumbing).

Activation convention: NHWC tensors of shape [n, h, w, c] whose channel dim is contiguous
(stride(3) == 1) and whose pixels are evenly strided (stride(2) = ld >= c, stride(1) = w*ld,
stride(0) = h*w*ld). A channel slice ``x[..., a:b]`` of such a tensor is again valid, which
is how the reference's torch.cat / channel slicing is expressed without copies.
Token tensors for linear layers are [rows, c] with stride(1) == 1.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import threading
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib
from ._lib import ConvDesc, call

NONE, LEAKY, GELU, SILU = 0, 1, 2, 3


def dt_code(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError(f"unsupported activation dtype {t.dtype}")


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def pix_ld(x: torch.Tensor) -> int:
    """Pixel stride of an NHWC activation (validates the layout)."""
    if x.dim() != 4 or x.stride(3) != 1:
        raise ValueError(f"expected NHWC activation with contiguous channels, got shape {tuple(x.shape)} "
                         f"strides {x.stride()}")
    n, h, w, c = x.shape
    ld = x.stride(2)
    if ld < c or (h > 1 and x.stride(1) != w * ld) or (n > 1 and x.stride(0) != h * w * ld):
        raise ValueError(f"activation pixels not evenly strided: shape {tuple(x.shape)} strides {x.stride()}")
    return ld


def new_act(n: int, h: int, w: int, c: int, dtype, device=None) -> torch.Tensor:
    return torch.empty((n, h, w, c), dtype=dtype, device=device or "cuda")


@dataclass
class ConvParams:
    """A conv / linear layer packed for rdeic_conv2d: weight [cout][wld] (K = (ky, kx, ci))."""
    weight: torch.Tensor
    wld: int
    bias: Optional[torch.Tensor]
    cout: int
    cin: int
    kh: int
    kw: int
    stride: int = 1
    pad: int = 0
    ln_cs: Optional[torch.Tensor] = None  # folded LayerNorm (ParamStore.conv_ln): column sums of the packed weight

    @staticmethod
    def pack(w: torch.Tensor, b: Optional[torch.Tensor], stride: int = 1, pad: int = 0,
             dtype=torch.bfloat16) -> "ConvParams":
        """Pack an fp32 torch-layout weight ([cout, cin, kh, kw] or Linear [cout, cin]) on device."""
        if w.dim() == 2:
            w = w[:, :, None, None]
        w = w.detach().to(device="cuda", dtype=torch.float32).contiguous()
        cout, cin, kh, kw = w.shape
        wld = ((kh * kw * cin + 63) // 64) * 64
        packed = torch.empty((cout, wld), dtype=dtype, device="cuda")
        call("rdeic_pack_conv_weight", w.data_ptr(), cout, cin, kh, kw, packed.data_ptr(), wld,
             1 if dtype == torch.bfloat16 else 0, stream_ptr())
        bias = None if b is None else b.detach().to(device="cuda", dtype=torch.float32).contiguous()
        return ConvParams(packed, wld, bias, cout, cin, kh, kw, stride, pad)


def conv2d(x: torch.Tensor, p: ConvParams, *, x2: Optional[torch.Tensor] = None, up2: bool = False,
           pad_t: Optional[int] = None, pad_l: Optional[int] = None, out_hw=None,
           gn: Optional[torch.Tensor] = None, gn_silu: bool = False, emb: Optional[torch.Tensor] = None,
           act: int = NONE, slope: float = 0.0, res: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, out_f32: bool = False, pixel_shuffle: bool = False,
           geglu: bool = False, stats: bool = False, stats_hw: Optional[int] = None,
           images: Optional[int] = None, ln_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = act(conv(cat(x, x2)) + bias + emb) + res   (all NHWC).
    images: how many images the launch covers when that is not n (token rows of ops.linear); the
    inference split-K count is chosen per image (SPLITK_NOMINAL_BATCH).
    geglu: p packed by ParamStore.conv_geglu; out = value * gelu(gate), cout/2 channels (bf16).
    stats: the output feeds a GroupNorm — its statistics are produced with it (fused into the conv
    epilogue where the tile allows, rdeic_conv_desc.gn_part) and group_norm_ab(out) then needs no
    pass over the tensor. stats_hw: pixels per image of that GroupNorm (default ho*wo).
    ln_rows: [M, 2] fp32 (mean, rstd) of the raw input rows from layer_norm_rowstats, with p packed by
    ParamStore.conv_ln: the output is linear(LayerNorm(x)) (the LayerNorm folded into the GEMM)."""
    if gn is not None and _gn_materialize(x, x2, p) and not _halo_eligible(x, x2, p, up2, pad_t, pad_l, out_hw,
                                                                           geglu or pixel_shuffle, out) \
            and not _edge_narrow_eligible(x, x2, p, up2, pad_t, pad_l, out_hw, geglu or pixel_shuffle or emb is not None):
        # the big-tile conv path has no GroupNorm prologue (it is VALU-bound there): materialise the
        # normalised (concatenated) input once with the vectorised, HBM-rate apply kernel instead
        xin = torch.empty(x.shape[:3] + (p.cin,), dtype=x.dtype, device=x.device)
        c0 = x.shape[3]
        pend = getattr(gn, "_rdeic_pending", None)
        if pend is not None and c0 % 8 == 0 and pix_ld(x) % 8 == 0 and x.data_ptr() % 16 == 0 and \
                (x2 is None or (x2.shape[3] % 8 == 0 and pix_ld(x2) % 8 == 0 and x2.data_ptr() % 16 == 0)):
            p0, pc0, p1, c1, n_, hw_, groups, eps, gamma, beta = pend
            _launch(("gn_apply", float(2 * xin.numel() * xin.element_size()), None), "rdeic_groupnorm_parts_apply",
                    p0.data_ptr(), pc0, _ptr(p1), c1, x.data_ptr(), pix_ld(x), _ptr(x2),
                    pix_ld(x2) if x2 is not None else 0, n_, hw_, groups, float(eps), gamma.data_ptr(),
                    beta.data_ptr(), int(gn_silu), gn.data_ptr(), xin.data_ptr(), pix_ld(xin), stream_ptr())
            del gn._rdeic_pending
        else:
            group_norm_apply(x, gn, gn_silu, out=xin[..., :c0])
            if x2 is not None:
                group_norm_apply(x2, gn[:, c0:], gn_silu, out=xin[..., c0:])
        x, x2, gn = xin, None, None
    n, h, w, c0 = x.shape
    ld0 = pix_ld(x)
    c1, ld1 = 0, 0
    if x2 is not None:
        if x2.shape[:3] != x.shape[:3] or x2.dtype != x.dtype:
            raise ValueError("concat inputs must share n, h, w and dtype")
        c1 = x2.shape[3]
        ld1 = pix_ld(x2)
    if c0 + c1 != p.cin:
        raise ValueError(f"conv expects cin={p.cin}, got {c0}+{c1}")
    if p.weight.dtype != x.dtype:
        raise TypeError(f"weight dtype {p.weight.dtype} != activation dtype {x.dtype}")
    hi, wi = (2 * h, 2 * w) if up2 else (h, w)
    pt = p.pad if pad_t is None else pad_t
    pl = p.pad if pad_l is None else pad_l
    if out_hw is None:
        ho = (hi + 2 * p.pad - p.kh) // p.stride + 1
        wo = (wi + 2 * p.pad - p.kw) // p.stride + 1
    else:
        ho, wo = out_hw
    odt = torch.float32 if (out_f32 or x.dtype == torch.float32) else x.dtype
    if geglu:
        if x.dtype != torch.bfloat16 or c0 % 64 or c1 % 64 or p.cout % 8 or res is not None or emb is not None \
                or act != NONE or out_f32 or pixel_shuffle:
            raise ValueError("fused GEGLU: bf16, 64-channel-aligned input, no residual / emb / activation")
        oshape = (n, ho, wo, p.cout // 2)
    elif pixel_shuffle:
        oshape = (n, 2 * ho, 2 * wo, p.cout // 4)
    else:
        oshape = (n, ho, wo, p.cout)
    if out is None:
        out = torch.empty(oshape, dtype=odt, device=x.device)
    elif tuple(out.shape) != oshape or out.dtype != odt:
        raise ValueError(f"out has shape {tuple(out.shape)}/{out.dtype}, expected {oshape}/{odt}")
    d = ConvDesc()
    d.in0 = x.data_ptr()
    d.in1 = _ptr(x2)
    d.c0, d.c1, d.ld0, d.ld1 = c0, c1, ld0, ld1
    d.n, d.h, d.w, d.up2 = n, h, w, int(up2)
    d.weight, d.wld, d.bias = p.weight.data_ptr(), p.wld, _ptr(p.bias)
    d.cout, d.kh, d.kw, d.stride, d.pad_t, d.pad_l = p.cout, p.kh, p.kw, p.stride, pt, pl
    d.ho, d.wo = ho, wo
    if gn is not None:
        if gn.shape != (n, p.cin, 2):
            raise ValueError("gn affine must be [n, cin, 2]")
        _ab_ready(gn)
        d.gn_ab = gn.data_ptr()
        d.gn_silu = int(gn_silu)
    if emb is not None:
        if emb.dtype != torch.float32 or emb.shape[0] != n or emb.stride(1) != 1:
            raise ValueError("emb must be fp32 [n, >=cout] row-major")
        d.emb = emb.data_ptr()
        d.emb_ld = emb.stride(0)
    d.act, d.act_param = act, float(slope)
    if res is not None:
        if tuple(res.shape) != oshape or res.dtype != odt:
            raise ValueError(f"residual {tuple(res.shape)}/{res.dtype} does not match output {oshape}/{odt}")
        d.res = res.data_ptr()
        d.res_ld = pix_ld(res)
    d.out = out.data_ptr()
    d.out_ld = pix_ld(out)
    d.out_mode = 2 if geglu else (1 if pixel_shuffle else 0)
    d.dtype = dt_code(x)
    d.out_f32 = int(odt == torch.float32 and x.dtype != torch.float32)
    d.batch = 1
    if ln_rows is not None:
        if p.ln_cs is None or ln_rows.dtype != torch.float32 or tuple(ln_rows.shape) != (n * ho * wo, 2) \
                or not ln_rows.is_contiguous():
            raise ValueError("ln_rows needs a ParamStore.conv_ln weight and an fp32 [M, 2] contiguous (mean, rstd)")
        d.ln_rows, d.ln_colsum = ln_rows.data_ptr(), p.ln_cs.data_ptr()
    elif p.ln_cs is not None:
        raise ValueError("a LayerNorm-folded weight needs ln_rows")
    part = None
    if stats and GN_STATS_FUSE and x.dtype == torch.bfloat16 and not (geglu or pixel_shuffle):
        ghw = int(stats_hw or ho * wo)
        nf = int(_lib.load().rdeic_groupnorm_parts_floats(n * ho * wo, p.cout, ghw))
        if nf:  # 0: the image size is not a multiple of 64 pixels; the GroupNorm reads the tensor
            part = torch.empty(nf, dtype=torch.float32, device=x.device)
            d.gn_part, d.gn_hw = part.data_ptr(), ghw
    flops = 2.0 * n * ho * wo * p.cout * p.kh * p.kw * p.cin
    splits = _splitk_count(x, x2, n * ho * wo, p, gn is not None or pixel_shuffle or geglu, out,
                           n if images is None else images)

    tile = -1
    if splits == 1 and x.dtype == torch.bfloat16 and gn is None and _gn_materialize(x, x2, p):
        key = tile_key(n * ho * wo, c0, c1, p, up2, d.out_mode, res is not None, emb is not None, act, odt)
        tile = TILE_TABLE.get(key, -1) if FORCE_TILE is None else FORCE_TILE
        if AUTOTUNE and FORCE_TILE is None and key not in TILE_TABLE:  # tuning runs only (tools/tune_tiles.py)
            # scratch with the output's exact strides (out may be a channel slice of a wider buffer)
            scratch = torch.empty_strided(out.size(), out.stride(), dtype=out.dtype, device=out.device)
            dma = c0 % 64 == 0 and c1 % 64 == 0
            tile = _autotune_tile(d, scratch, DMA_TILE_CANDIDATES if dma else TILE_CANDIDATES)
            if tile >= 0:
                TILE_TABLE[key] = tile

    tag = ("conv", flops, (n, h, w, c0, c1, p.cout, p.kh, p.stride, gn is not None, int(up2), d.out_mode))
    if splits > 1:
        ws = _splitk_workspace(splits * n * ho * wo * p.cout, x.device)
        _launch(tag, "rdeic_conv2d_splitk", C.byref(d), splits, ws.data_ptr(), ws.numel(), stream_ptr())
    elif tile >= 0:
        _launch(tag, "rdeic_conv2d_tile", C.byref(d), tile, stream_ptr())
    else:
        _launch(tag, "rdeic_conv2d", C.byref(d), stream_ptr())
    if part is not None:
        _attach_gn_part(out, part, d.gn_hw)
    return out


# Fused GroupNorm statistics (conv2d(stats=True) -> group_norm_ab): the partial sums travel as an
# attribute of the output tensor object, keyed on its storage and shape, so a view or a different
# tensor never picks up another tensor's statistics (it simply takes the stand-alone stats pass).
GN_STATS_FUSE = True


def _attach_gn_part(t: torch.Tensor, part: torch.Tensor, hw: int) -> None:
    t._rdeic_gn_part = (part, t.data_ptr(), tuple(t.shape), tuple(t.stride()), hw)


def _gn_part_of(t: Optional[torch.Tensor], hw: int):
    info = getattr(t, "_rdeic_gn_part", None) if t is not None else None
    if info is None:
        return None
    part, ptr, shape, stride, phw = info
    if ptr != t.data_ptr() or shape != tuple(t.shape) or stride != tuple(t.stride()) or phw != hw:
        return None
    return part


# Tile choice for the big-tile bf16 conv path. Every tile produces bit-identical results (same BK,
# same MFMA, same k order; tests/test_tiles_gpu.py runs every tile id on every layer-shape class
# against the default), so the choice only changes speed. It comes from a COMMITTED per-shape table
# (conv_tiles.json, measured once on an MI355X by tools/tune_tiles.py): the same kernel runs for a
# given shape in every process and on every box. Shapes missing from the table use the library's
# built-in heuristic (tile -1). AUTOTUNE (tuning runs only) times the candidates for missing shapes.
# Layers whose channel segments are multiples of 64 run on the LDS-DMA kernel (tile ids 21..38,
# rdeic_hip.h); the others on the register-staged tiles (0..10).
AUTOTUNE = False
FORCE_TILE: Optional[int] = None  # tests / tools: run every eligible conv on this tile id
GEGLU_FUSED = True  # bf16 transformer FF: GEGLU in the projection's epilogue (conv out_mode 2)
TILE_CANDIDATES = (0, 1, 3, 4, 6, 8, 10)
DMA_TILE_CANDIDATES = (25, 32, 34, 26, 30, 33, 24, 31, 35, 36, 37, 38)
ALL_TILES = (0, 1, 2, 3, 4, 6, 7, 8, 9, 10) + tuple(range(21, 39))
# RDEIC_TILE_TABLE: another table file (same-box A/B of tile tables, tools/table_ab.sh)
TILE_TABLE_PATH = os.environ.get("RDEIC_TILE_TABLE") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                                     "conv_tiles.json")


def tile_key(m: int, c0: int, c1: int, p: "ConvParams", up2: bool, out_mode: int, res: bool, emb: bool, act: int,
             odt) -> str:
    """Layer-shape key of the tile table: GEMM M, the concat split, filter, stride, fused epilogue."""
    return (f"m{m}:c{c0}+{c1}:o{p.cout}:k{p.kh}x{p.kw}:s{p.stride}:up{int(up2)}:om{out_mode}:"
            f"r{int(res)}:e{int(emb)}:a{act}:{'f32' if odt == torch.float32 else 'bf16'}")


def _load_tile_table() -> dict:
    if not os.path.exists(TILE_TABLE_PATH):
        return {}
    with open(TILE_TABLE_PATH) as f:
        tab = json.load(f)["tiles"]
    bad = {k: v for k, v in tab.items() if v not in ALL_TILES}
    if bad:
        raise ValueError(f"{TILE_TABLE_PATH}: unknown tile ids {bad}")
    return tab


TILE_TABLE: dict = _load_tile_table()


def _autotune_tile(d0, scratch: torch.Tensor, candidates=None) -> int:
    """Time each candidate writing into `scratch` (the real output may alias the residual)."""
    if _lib.RECORDER is not None:  # never record tuning launches: keep the heuristic choice
        return -1
    d = ConvDesc.from_buffer_copy(d0)
    d.out = scratch.data_ptr()
    s = stream_ptr()
    best, best_t = -1, float("inf")
    for t in (TILE_CANDIDATES if candidates is None else candidates):
        call("rdeic_conv2d_tile", C.byref(d), t, s)  # warm (first launch of a kernel variant)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(2):
            call("rdeic_conv2d_tile", C.byref(d), t, s)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        if ms < best_t:
            best, best_t = t, ms
    return best


# Split-K is opt-in (see splitk_allowed): it changes the k grouping, so layers whose outputs must
# be batch-invariant (the entropy-model nets) never use it. The switches are PER HOST THREAD: codec
# sessions run compress / decompress on their own threads, and one session leaving its split-K region
# must not turn split-K off under another session's entropy nets (their encoder and decoder would then
# compute different mu / sigma).
_SPLITK_WS: dict = {}
_SPLITK_TLS = threading.local()


def splitk_state():
    """(allowed, short_k) of the calling thread's split-K switches."""
    return getattr(_SPLITK_TLS, "allowed", False), getattr(_SPLITK_TLS, "short", False)


# Inference picks the split count from the layer's PER-IMAGE shape, as if the batch were
# SPLITK_NOMINAL_BATCH images (config 2's 16): the k grouping of every output element then does not
# depend on how many images share the launch, so one bitstream decodes to the same pixels in any
# batch (bench, CLI --batch_size / --micro_batch_size, data-parallel shards). Training (short_k,
# B=1) sizes splits from the real M: it needs no batch invariance.
SPLITK_NOMINAL_BATCH = 16
# Inference split rule: tiles x splits within SPLITK_BLOCKS co-resident 128x128 blocks, at most SPLITK_MAX splits
# (A/B knobs: bench.py --splitk-rule BLOCKS,MAX; a change moves the k grouping and so the bf16 rounding of the
# split layers, the entropy nets' too: both codec sides apply the same rule, so bitstreams stay self-consistent)
SPLITK_BLOCKS, SPLITK_MAX = 512, 8
# Training (short_k) split counts for the >= 32 k-tile layers: None = the inference rule below; else
# (k-tiles per split at least, max splits, target blocks) -- an A/B knob (bench_train.py --splitk-train)
SPLITK_TRAIN = None
# bf16 entropy model (Compression nets at the y / z resolution): split-K allowed, per-image counts
SPLITK_ENTROPY = True


class splitk_allowed:
    """Context manager enabling split-K for small-M / large-K convs (UNet / control forward) on the
    calling thread. short_k (the fine-tune step, B=1): also split layers with as few as 8 k-tiles."""

    def __init__(self, short_k: bool = False):
        self.short_k = short_k

    def __enter__(self):
        self._prev = splitk_state()
        _SPLITK_TLS.allowed, _SPLITK_TLS.short = True, self.short_k or self._prev[1]
        return self

    def __exit__(self, *exc):
        _SPLITK_TLS.allowed, _SPLITK_TLS.short = self._prev


class splitk_as:
    """Context manager restoring a captured splitk_state() on the calling thread. PyTorch runs the
    backward of autograd Functions on its own per-device engine thread, whose switches are the
    defaults (off): Conv2dFn / LinearFn capture the forward thread's state in ctx and re-enter it
    around their backward convs, so the input gradients of a training step split K as the forward
    did (finetune.py's splitk_allowed(short_k=True))."""

    def __init__(self, state):
        self.state = tuple(state)

    def __enter__(self):
        self._prev = splitk_state()
        _SPLITK_TLS.allowed, _SPLITK_TLS.short = self.state
        return self

    def __exit__(self, *exc):
        _SPLITK_TLS.allowed, _SPLITK_TLS.short = self._prev


def _splitk_count(x, x2, M: int, p: "ConvParams", fused: bool, out: torch.Tensor, n: int) -> int:
    """Number of k-splits (1 = none): only when the 128x128 tile grid cannot fill the chip.
    Inference: a function of the per-image M only (SPLITK_NOMINAL_BATCH); n = images in the launch."""
    allowed, short = splitk_state()
    if not short:
        M = (M // max(1, n)) * SPLITK_NOMINAL_BATCH
    if not allowed or fused or x.dtype not in (torch.bfloat16, torch.float32) or p.cout % 8 \
            or pix_ld(out) % 8 or out.data_ptr() % 16:
        return 1
    for t in (x, x2):
        if t is not None and (t.shape[3] % 8 or pix_ld(t) % 8 or t.data_ptr() % 16):
            return 1
    if x.dtype == torch.float32:  # 64x64 fp32 tiles, 32-deep k-steps
        tiles = -(-M // 64) * -(-p.cout // 64)
        nk = -(-(p.kh * p.kw * p.cin) // 32)
        if short and tiles < 256 and 8 <= nk < 32:
            return max(1, min(-(-512 // tiles), nk // 4, 16))
        if tiles >= 256 or nk < 32:
            return 1
        return max(1, min(-(-512 // tiles), nk // 8, 16))
    tiles = -(-M // 128) * -(-p.cout // 128)
    nk = -(-(p.kh * p.kw * p.cin) // 64)
    if short and tiles < 128 and 8 <= nk < 32:
        return max(1, min(-(-512 // tiles), nk // 4, 8))
    if short and SPLITK_TRAIN is not None and tiles < 192 and nk >= 32:  # A/B knob (bench_train.py --splitk-train)
        kdiv, smax, target = SPLITK_TRAIN
        return max(1, min(-(-target // tiles), nk // kdiv, smax))
    if tiles >= 192 or nk < 32:
        return 1
    # tiles x splits within the 512 co-resident 128x128 blocks (2 per CU): one more split past that
    # starts a second round of blocks (tools/splitk_bench.py, UNet 8x8 level: 7 splits 419 / 503 TF,
    # 6 splits 528 / 674 TF for the 1280 / 2560-channel inputs)
    return max(1, min(SPLITK_BLOCKS // tiles, nk // 16, SPLITK_MAX))


_SPLITK_KEEP: list = []  # every workspace ever handed out: recorded launch plans hold their pointers


def _splitk_workspace(n: int, device) -> torch.Tensor:
    """Split-K partial-sum scratch, one per (device, stream): concurrent codec sessions (one per
    stream) must not share it. A grown workspace replaces the old one for new
    launches, but the old one stays allocated (plans recorded earlier still point at it)."""
    key = (str(device), stream_ptr())
    buf = _SPLITK_WS.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.empty(n, dtype=torch.float32, device=device)
        _SPLITK_WS[key] = buf
        _SPLITK_KEEP.append(buf)
    return buf


# When set to a list, every rdeic_conv2d launch appends (algorithmic FLOPs, start event, end
# event, dtype) — bench.py uses it to time the dominant kernel live over its timed region.
# The secondary kernels (attention: FLOPs; GroupNorm statistics / apply: algorithmic bytes) go to
# PROFILE_OTHER[kind] as (work, start event, end event) while PROFILE is set.
PROFILE = None
PROFILE_OTHER: dict = {}


def _launch(tag, name: str, *args):
    """call(name, *args); when profiling, bracket it with events on the current stream and file it
    under tag = (kind, work, meta): "conv" -> PROFILE, anything else -> PROFILE_OTHER[kind]."""
    if PROFILE is None:
        return call(name, *args, tag=tag)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record()
    call(name, *args, tag=tag)
    ev1.record()
    record_profile(tag, ev0, ev1)


def record_profile(tag, ev0, ev1):
    kind, work, meta = tag
    if kind == "conv":
        PROFILE.append((work, ev0, ev1, None, meta))
    else:
        PROFILE_OTHER.setdefault(kind, []).append((work, ev0, ev1))


PROF_KINDS = {"conv": 0, "attention": 1, "attention_dh16": 2, "gn_stats": 3, "gn_apply": 4, "gemm": 5,
              "attention_d512": 6, "conv_bytes": 7}


def prof_start(capacity: int = 65536, every: int = 1) -> None:
    """Native launch profiler (rdeic_prof_*): the launchers record HIP events on their stream,
    for one launch in `every` of each kind."""
    call("rdeic_prof_start", capacity, every)


def prof_stop() -> int:
    return int(_lib.load().rdeic_prof_stop())


def prof_read() -> dict:
    """{kind: (launches, algorithmic work, event-timed ms)} recorded since prof_start (synchronizes)."""
    out = {}
    for kind, code in PROF_KINDS.items():
        n, w, ms = C.c_int64(), C.c_double(), C.c_double()
        call("rdeic_prof_read", code, C.byref(n), C.byref(w), C.byref(ms))
        if n.value:
            out[kind] = (n.value, w.value, ms.value)
    return out


def prof_read_keys(kind: str, cap: int = 64) -> list:
    """[(key, launches, work, event ms)] per launch-shape key of one kind (rdeic_prof_read_keys; synchronizes)."""
    keys, n = (C.c_int64 * cap)(), (C.c_int64 * cap)()
    w, ms = (C.c_double * cap)(), (C.c_double * cap)()
    m = int(_lib.load().rdeic_prof_read_keys(PROF_KINDS[kind], keys, n, w, ms, cap))
    return [(int(keys[i]), int(n[i]), float(w[i]), float(ms[i])) for i in range(max(0, m))]


def attention_key(key: int) -> dict:
    """Decode an attention profiler key: head dim, query / key lengths, batch x heads."""
    return {"dh": (key >> 48) & 0xffff, "lq": (key >> 32) & 0xffff, "lk": (key >> 16) & 0xffff, "bh": key & 0xffff}


def other_profile_summary():
    """{kind: (launches, total work, total ms)} of the secondary kernels (after sync)."""
    out = {}
    for kind, recs in PROFILE_OTHER.items():
        out[kind] = (len(recs), sum(r[0] for r in recs), sum(r[1].elapsed_time(r[2]) for r in recs))
    return out


def conv_profile_summary(records):
    """(launches, total algorithmic FLOPs, total kernel ms) of recorded conv launches (after sync)."""
    total_ms = 0.0
    total_flops = 0.0
    for rec in records:
        flops, e0, e1 = rec[0], rec[1], rec[2]
        total_ms += e0.elapsed_time(e1)
        total_flops += flops
    return len(records), total_flops, total_ms


def conv_profile_breakdown(records):
    """{shape-class: [launches, GFLOP, ms]} for diagnosing where the conv time goes."""
    out = {}
    for rec in records:
        flops, e0, e1, meta = rec[0], rec[1], rec[2], rec[4]
        key = str(meta)
        v = out.setdefault(key, [0, 0.0, 0.0])
        v[0] += 1
        v[1] += flops / 1e9
        v[2] += e0.elapsed_time(e1)
    return out


CONV_PATH = 2  # mirrors rdeic_set_conv_path (0: fused-GN 128-tiles everywhere, 2: big-tile auto choice)


def set_conv_path(path: int) -> int:
    global CONV_PATH
    prev = CONV_PATH
    CONV_PATH = int(path)
    _lib.load().rdeic_set_conv_path(CONV_PATH)
    return prev


def set_conv_option(key: int, value: int) -> int:
    """rdeic_set_conv_option (include/rdeic_hip.h): 0 vector epilogue, 1 dh=64 attention kernel, 3 swizzle,
    4 forced register tile, 5 LDS-DMA path, 6 halo conv, 8 d=512 attention form, 9 8-row halo conv, 10 VAE edge
    convs."""
    return int(_lib.load().rdeic_set_conv_option(int(key), int(value)))


# 3x3 halo conv (rdeic_amd/csrc/conv_halo.hip, conv3x3_halo8_kernel / conv3x3_halo_kernel): a conv whose input is a
# GroupNorm (+ SiLU) of a single 32-channel-aligned NHWC tensor and whose output tiles as 4 x 64 pixel
# blocks x 128 channels takes the raw input and applies the affine once per element in LDS, instead
# of materialising the normalised tensor (rdeic_set_conv_option(6, .): 0 off, 1 GroupNorm inputs, 2 all).
HALO_CONV = 1
# widest input / output the halo conv takes over from the materialised path: measured at B=16
# (tools/halo_bench.py, r03) it wins on the 512^2 128-channel layers (2.14 -> 1.53 ms, 3.59 -> 2.62 ms)
# and the 256^2 ones (0.86 -> 0.75, 1.39 -> 1.26 ms) and ties the 256x256 im2col tiles on the
# 512-channel layers at 128^2 / 64^2 (where it still saves the GroupNorm apply launches)
HALO_MAX_C = 512


# launch counters of the library (rdeic_launch_count, RDEIC_COUNT_* in include/rdeic_hip.h)
COUNT_HALO_CONV, COUNT_GN_APPLY, COUNT_LAYERNORM, COUNT_HALO_SMALL, COUNT_LN_FUSED, COUNT_SPLITK, COUNT_EDGE, \
    COUNT_GN_PARTS_APPLY = 0, 1, 2, 3, 4, 5, 6, 7


def launch_count(kind: int) -> int:
    """Launches of one kernel family since the last launch_count_reset (host-side counter)."""
    return int(_lib.load().rdeic_launch_count(int(kind)))


def launch_count_reset() -> None:
    call("rdeic_launch_count_reset")


def set_halo_conv(mode: int) -> int:
    global HALO_CONV
    prev = HALO_CONV
    HALO_CONV = int(mode)
    _lib.load().rdeic_set_conv_option(6, HALO_CONV)
    return prev


def _halo_eligible(x, x2, p: "ConvParams", up2, pad_t, pad_l, out_hw, special, out) -> bool:
    """Mirror of the library's halo_ok (the conv2d_run dispatch) for a GroupNorm-input conv."""
    if not HALO_CONV or x.dtype != torch.bfloat16 or x2 is not None or up2 or special:
        return False
    if p.kh != 3 or p.kw != 3 or p.stride != 1 or p.pad != 1 or (pad_t not in (None, 1)) or (pad_l not in (None, 1)):
        return False
    n, h, w, c = x.shape
    if out_hw is not None and tuple(out_hw) != (h, w):
        return False
    if c % 32 or c > min(512, HALO_MAX_C) or p.cout > HALO_MAX_C or p.cout % 128 or h % 4 or w % 64 \
            or x.stride(2) % 8 or x.data_ptr() % 16:
        return False
    if out is not None and (pix_ld(out) % 8 or out.data_ptr() % 16):
        return False
    return True


# The VAE edge convs (rdeic_amd/csrc/conv_edge.hip, rdeic_set_conv_option(10, .)): conv_in from 8 channels on
# direct-load MFMA fragments, and norm -> SiLU -> 3x3 conv to <= 16 channels (the decoder's conv_out) with the
# GroupNorm applied once per element in LDS instead of materialised (one read of the input instead of read + write
# + read).
EDGE_CONV = 1


def set_edge_conv(mode: int) -> int:
    global EDGE_CONV
    prev = EDGE_CONV
    EDGE_CONV = int(mode)
    _lib.load().rdeic_set_conv_option(10, EDGE_CONV)
    return prev


def _edge_narrow_eligible(x, x2, p: "ConvParams", up2, pad_t, pad_l, out_hw, special) -> bool:
    """Mirror of the library's launch_edge rule for the GroupNorm-input narrow conv."""
    if not EDGE_CONV or x.dtype != torch.bfloat16 or x2 is not None or up2 or special:
        return False
    if p.kh != 3 or p.kw != 3 or p.stride != 1 or p.pad != 1 or (pad_t not in (None, 1)) or (pad_l not in (None, 1)):
        return False
    n, h, w, c = x.shape
    if out_hw is not None and tuple(out_hw) != (h, w):
        return False
    lds = 10 * 66 * 64 + c * 8 + p.cout * 9 * c * 2  # 8-row halo, GroupNorm table, weights (conv_edge.hip)
    return p.cout <= 16 and c % 32 == 0 and lds <= 160 * 1024 and h % 8 == 0 and w % 64 == 0 \
        and x.stride(2) % 8 == 0 and x.data_ptr() % 16 == 0


def _gn_materialize(x: torch.Tensor, x2: Optional[torch.Tensor], p: ConvParams) -> bool:
    """Same rule as rdeic_conv2d's dispatch to the big-tile path (bf16, 16-byte gathers, cout > 32), plus
    the large tiny-cout convs (the VAE's conv_out): their direct kernel would redo the GroupNorm + SiLU
    of every input element for all 9 taps."""
    if CONV_PATH == 0 or x.dtype != torch.bfloat16:
        return False
    if p.cout <= 32 and not (p.cout <= 4 and x.shape[0] * x.shape[1] * x.shape[2] >= (1 << 20)):
        return False
    for t in (x, x2):
        if t is None:
            continue
        if t.shape[3] % 8 or t.stride(2) % 8 or t.data_ptr() % 16:
            return False
    return True


def linear(x: torch.Tensor, p: ConvParams, *, act: int = NONE, res: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, out_f32: bool = False, geglu: bool = False,
           stats_hw: Optional[int] = None, images: int, ln_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Token-wise Linear over a [rows, c] tensor (1x1 conv over a rows x 1 image).
    images: the number of images whose tokens the rows hold (required: the per-image split-K choice
    keeps every output's k grouping independent of the batch).
    geglu: fused GEGLU projection (p from ParamStore.conv_geglu), output [rows, cout/2].
    stats_hw: the output (as [rows/stats_hw images, stats_hw tokens]) feeds a GroupNorm; its
    statistics are produced with it (conv2d(stats=True)); reshape with ops.tokens_to_nhwc."""
    rows, c = x.shape
    x4 = x.as_strided((1, rows, 1, c), (rows * x.stride(0), x.stride(0), x.stride(0), 1))
    odt = torch.float32 if (out_f32 or x.dtype == torch.float32) else x.dtype
    cw = p.cout // 2 if geglu else p.cout
    if out is None:
        out = torch.empty((rows, cw), dtype=odt, device=x.device)
    o4 = out.as_strided((1, rows, 1, cw), (rows * out.stride(0), out.stride(0), out.stride(0), 1))
    r4 = None
    if res is not None:
        r4 = res.as_strided((1, rows, 1, p.cout), (rows * res.stride(0), res.stride(0), res.stride(0), 1))
    conv2d(x4, p, act=act, res=r4, out=o4, out_f32=out_f32, geglu=geglu, stats=stats_hw is not None,
           stats_hw=stats_hw, images=images, ln_rows=ln_rows)
    info = getattr(o4, "_rdeic_gn_part", None)
    if info is not None:
        out._rdeic_gn_tokens = info  # carried to the NHWC view by tokens_to_nhwc
    return out


def tokens_to_nhwc(t: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    """[n*h*w, c] token rows -> NHWC view, keeping fused GroupNorm statistics of linear(stats_hw=h*w)."""
    v = t.view(n, h, w, t.shape[1])
    info = getattr(t, "_rdeic_gn_tokens", None)
    if info is not None and info[4] == h * w:
        _attach_gn_part(v, info[0], h * w)
    return v


def gemm_batched(a: torch.Tensor, b_nk: torch.Tensor, out: torch.Tensor, *, batch: int, m: int, n: int, k: int,
                 lda: int, ldb: int, a_bs: int, b_bs: int, out_bs: int) -> torch.Tensor:
    """out[z] (m x n, row stride n) = A[z] (m x k, row stride lda) . B[z]^T (B stored n x k, row stride ldb).
    ldb must be a multiple of 64 and B zero beyond k (it is used as a packed weight)."""
    d = ConvDesc()
    d.in0 = a.data_ptr()
    d.c0, d.ld0 = k, lda
    d.n, d.h, d.w = 1, m, 1
    d.weight, d.wld = b_nk.data_ptr(), ldb
    d.cout, d.kh, d.kw, d.stride = n, 1, 1, 1
    d.ho, d.wo = m, 1
    d.out = out.data_ptr()
    d.out_ld = n
    d.dtype = dt_code(a)
    d.out_f32 = int(out.dtype == torch.float32 and a.dtype != torch.float32)
    d.batch = batch
    d.in_bs, d.w_bs, d.out_bs = a_bs, b_bs, out_bs
    _launch(("conv", 2.0 * batch * m * n * k, ("bgemm", batch, m, n, k)), "rdeic_conv2d", C.byref(d), stream_ptr())
    return out


# GroupNorm finalize + apply in ONE launch on small images (rdeic_groupnorm_parts_apply: the UNet / control net's
# 16^2 and 8^2 levels, where the finalize and the apply are each a ~10 us latency floor). group_norm_ab(...,
# defer=True) then returns the affine with its finalize pending; conv2d's materialised GroupNorm runs the fused
# launch (which also fills the affine), and any other consumer of the affine finalizes it first (_ab_ready).
GN_PARTS_APPLY = True
GN_PARTS_APPLY_HW = (64, 128, 256)


def _ab_ready(ab: Optional[torch.Tensor]) -> None:
    """Run a deferred GroupNorm finalize (group_norm_ab(defer=True)) before the affine is read."""
    pend = getattr(ab, "_rdeic_pending", None) if ab is not None else None
    if pend is None:
        return
    p0, c0, p1, c1, n, hw, groups, eps, gamma, beta = pend
    call("rdeic_groupnorm_parts_ab", p0.data_ptr(), c0, _ptr(p1), c1, n, hw, groups, float(eps),
         gamma.data_ptr(), beta.data_ptr(), ab.data_ptr(), stream_ptr())
    del ab._rdeic_pending


def group_norm_ab(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, groups: int, eps: float,
                  x2: Optional[torch.Tensor] = None, defer: bool = False) -> torch.Tensor:
    """Per-(image, channel) affine [n, c, 2] such that GroupNorm(cat(x, x2)) = x*a + b.
    defer: the caller hands the affine straight to conv2d(gn=...): on small images with fused statistics its
    finalize is left pending and runs inside that conv's materialised GroupNorm (rdeic_groupnorm_parts_apply)."""
    n, h, w, c0 = x.shape
    ld0 = pix_ld(x)
    c1, ld1 = (x2.shape[3], pix_ld(x2)) if x2 is not None else (0, 0)
    c = c0 + c1
    p0, p1 = _gn_part_of(x, h * w), _gn_part_of(x2, h * w)
    if p0 is not None and (x2 is None or p1 is not None):
        # statistics came with the producing conv: only the per-(image, group) finalize runs
        ab = torch.empty((n, c, 2), dtype=torch.float32, device=x.device)
        if defer and GN_PARTS_APPLY and h * w in GN_PARTS_APPLY_HW and x.dtype == torch.bfloat16 and groups <= 256:
            ab._rdeic_pending = (p0, c0, p1, c1, n, h * w, groups, float(eps), gamma, beta)
            return ab
        call("rdeic_groupnorm_parts_ab", p0.data_ptr(), c0, _ptr(p1), c1, n, h * w, groups, float(eps),
             gamma.data_ptr(), beta.data_ptr(), ab.data_ptr(), stream_ptr())
        return ab
    ws = torch.empty(int(_lib.load().rdeic_groupnorm_ws_floats(n, h * w, c)), dtype=torch.float32, device=x.device)
    ab = torch.empty((n, c, 2), dtype=torch.float32, device=x.device)
    _launch(("gn_stats", float(n * h * w * c * x.element_size()), None),
            "rdeic_groupnorm_stats", x.data_ptr(), c0, ld0, _ptr(x2), c1, ld1, n, h * w, groups,
            float(eps), gamma.data_ptr(), beta.data_ptr(), ab.data_ptr(), ws.data_ptr(), dt_code(x), stream_ptr())
    return ab


def group_norm_apply(x: torch.Tensor, ab: torch.Tensor, silu: bool, out: Optional[torch.Tensor] = None,
                     out_mul: float = 1.0) -> torch.Tensor:
    """y = silu?(x*a + b) * out_mul; `ab` may be a channel slice ab[:, c0:] of a wider affine."""
    _ab_ready(ab)
    n, h, w, c = x.shape
    if out is None:
        out = torch.empty((n, h, w, c), dtype=x.dtype, device=x.device)
    if ab.shape[1] < c or ab.stride(2) != 1 or ab.stride(1) != 2:
        raise ValueError("group-norm affine must be [n, >=c, 2] with packed (a, b) pairs")
    _launch(("gn_apply", float(2 * n * h * w * c * x.element_size()), None),
            "rdeic_groupnorm_apply", x.data_ptr(), n, h * w, c, pix_ld(x), ab.data_ptr(),
            ab.stride(0) // 2, int(silu), float(out_mul), out.data_ptr(), pix_ld(out), dt_code(x), stream_ptr())
    return out


# bf16 transformer LayerNorms folded into the consuming linear (rdeic_layernorm_rowstats + conv_ln weights):
# the normalised tensor is never written
LN_FOLD = True


def layer_norm_rowstats(x: torch.Tensor, eps: float = 1e-5, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[rows, c] bf16 -> [rows, 2] fp32 (mean, 1/sqrt(var + eps)) per row (torch.nn.LayerNorm's statistics)."""
    rows, c = x.shape
    if out is None:
        out = torch.empty((rows, 2), dtype=torch.float32, device=x.device)
    call("rdeic_layernorm_rowstats", x.data_ptr(), rows, c, x.stride(0), float(eps), out.data_ptr(), stream_ptr())
    return out


def layer_norm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    rows, c = x.shape
    if out is None:
        out = torch.empty((rows, c), dtype=x.dtype, device=x.device)
    call("rdeic_layernorm", x.data_ptr(), rows, c, x.stride(0), gamma.data_ptr(), beta.data_ptr(), float(eps),
         out.data_ptr(), out.stride(0), dt_code(x), stream_ptr())
    return out


def attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: torch.Tensor, *, batch: int, heads: int,
              lq: int, lk: int, dh: int, scale: float, kv_bcast: bool = False) -> torch.Tensor:
    """Flash attention over [batch*lq, heads*dh]-layout projections (row strides from the tensors).
    kv_bcast: K/V hold one batch shared by every query batch."""
    _launch(("attention_d512" if dh == 512 else "attention" if dh >= 64 else "attention_dh%d" % dh,
             4.0 * batch * heads * lq * lk * dh, None),
            "rdeic_attention", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(),
            v.stride(0), out.data_ptr(), out.stride(0), batch, heads, lq, lk, dh, float(scale),
            int(kv_bcast), dt_code(q), stream_ptr())
    return out


# VAE AttnBlock in bf16 on the flash kernel (rdeic_attention, dh = 512); False: the materialised path
VAE_FLASH_ATTENTION = True

# Score-buffer budget of the single-head (VAE, d=512) attention: the fp32 scores of one query
# chunk never exceed it, so the buffer is O(chunk x L), not O(B x L^2). At 1024x1024 one image's
# full score matrix would be 16384^2 x 4 B = 1 GiB: it runs as 4 query-row chunks of 4096 rows.
# At 512x512 (64 MiB per image) a chunk holds 4 images.
SCORE_BUDGET_BYTES = 1 << 28


def attention_single_head_materialized(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, out: torch.Tensor, *,
                                       batch: int, length: int, dim: int, scale: float) -> torch.Tensor:
    """softmax(q k^T * scale) v for one head with a large head dim (VAE AttnBlock, d=512,
    model.py:181-205): per chunk of query rows (whole images while they fit the score budget,
    else row blocks of one image), S = Q K^T (batched MFMA GEMM, fp32) -> row softmax -> O = P V
    (batched GEMM). Every output row is computed exactly as without chunking (same k order)."""
    if dim % 64 != 0 or length % 64 != 0:
        raise ValueError("materialised attention needs dim, length multiples of 64")
    dt = dt_code(q)
    L = length
    per_img = L * L * 4
    if per_img <= SCORE_BUDGET_BYTES:
        g, qrows = max(1, min(batch, SCORE_BUDGET_BYTES // per_img)), L
    else:
        g, qrows = 1, max(64, (SCORE_BUDGET_BYTES // (L * 4)) // 64 * 64)
    vt = torch.empty((batch, dim, L), dtype=q.dtype, device=q.device)
    call("rdeic_transpose", v.data_ptr(), L, dim, v.stride(0), vt.data_ptr(), L, batch,
         L * v.stride(0), dim * L, dt, stream_ptr())
    s = torch.empty((g, qrows, L), dtype=torch.float32, device=q.device)
    p = torch.empty((g, qrows, L), dtype=q.dtype, device=q.device)
    for b0 in range(0, batch, g):
        nb = min(g, batch - b0)
        for q0 in range(0, L, qrows):
            nq = min(qrows, L - q0)
            qa = q[b0 * L + q0:]
            gemm_batched(qa, k[b0 * L:], s, batch=nb, m=nq, n=L, k=dim, lda=q.stride(0), ldb=k.stride(0),
                         a_bs=L * q.stride(0), b_bs=L * k.stride(0), out_bs=nq * L)
            call("rdeic_softmax_rows", s.data_ptr(), nb * nq, L, float(scale), p.data_ptr(), dt, stream_ptr())
            gemm_batched(p, vt[b0:], out[b0 * L + q0:], batch=nb, m=nq, n=dim, k=L, lda=L, ldb=L,
                         a_bs=nq * L, b_bs=dim * L, out_bs=L * out.stride(0))
    return out


def geglu(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    rows, c2 = x.shape
    c = c2 // 2
    if out is None:
        out = torch.empty((rows, c), dtype=x.dtype, device=x.device)
    call("rdeic_geglu", x.data_ptr(), rows, c, x.stride(0), out.data_ptr(), out.stride(0), dt_code(x), stream_ptr())
    return out


def cfg_combine(e_cond: torch.Tensor, e_uncond: torch.Tensor, scale: float) -> torch.Tensor:
    """Classifier-free guidance e_u + scale * (e_c - e_u) (fp32, the reference's op order)."""
    if e_cond.dtype != torch.float32 or e_uncond.dtype != torch.float32 or e_cond.shape != e_uncond.shape:
        raise ValueError("cfg_combine needs two fp32 tensors of one shape")
    ec, eu = e_cond.contiguous(), e_uncond.contiguous()
    out = torch.empty_like(ec)
    call("rdeic_cfg_combine", ec.data_ptr(), eu.data_ptr(), ec.numel(), float(scale), out.data_ptr(), stream_ptr())
    return out


def nchw_to_nhwc(x: torch.Tensor, dtype, mul: float = 1.0, add: float = 0.0, out=None) -> torch.Tensor:
    x = x.to(torch.float32).contiguous()
    n, c, h, w = x.shape
    if out is None:
        out = torch.empty((n, h, w, c), dtype=dtype, device=x.device)
    call("rdeic_nchw_to_nhwc", x.data_ptr(), n, c, h, w, float(mul), float(add), out.data_ptr(), pix_ld(out),
         dt_code(out), stream_ptr())
    return out


def nhwc_to_nchw(x: torch.Tensor, mul: float = 1.0, add: float = 0.0) -> torch.Tensor:
    n, h, w, c = x.shape
    out = torch.empty((n, c, h, w), dtype=torch.float32, device=x.device)
    call("rdeic_nhwc_to_nchw", x.data_ptr(), n, c, h, w, pix_ld(x), float(mul), float(add), out.data_ptr(),
         dt_code(x), stream_ptr())
    return out


def cast(x: torch.Tensor, dtype) -> torch.Tensor:
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=dtype, device=x.device)
    call("rdeic_cast", x.data_ptr(), dt_code(x), out.data_ptr(), dt_code(out), x.numel(), stream_ptr())
    return out


def fill_uniform(out: torch.Tensor, seed: int, scale: float, offset: float) -> torch.Tensor:
    if out.dtype != torch.float32 or not out.is_contiguous():
        raise ValueError("fill_uniform expects a contiguous fp32 tensor")
    call("rdeic_fill_uniform", out.data_ptr(), out.numel(), C.c_uint64(seed & 0xFFFFFFFFFFFFFFFF),
         float(scale) * 2.0 ** -23, float(offset), stream_ptr())
    return out


def silu_f32(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(x)
    call("rdeic_silu_f32", x.data_ptr(), out.data_ptr(), x.numel(), stream_ptr())
    return out
