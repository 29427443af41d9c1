"""Differentiable ops of the adapter fine-tune step (config 5), each a torch.autograd.Function whose
forward AND backward run on the HIP kernels of librdeic_hip.so (train.hip, conv_gemm.hip, norm.hip,
attention.hip). torch's autograd engine only sequences them and accumulates gradients.

Layout: activations NHWC (channel-contiguous, pixel stride ld), token tensors [rows, c] with a row
stride; weights are the fp32 masters in torch layout ([cout, cin, kh, kw] / [cout, cin]) so weight
gradients land where torch.optim / the reference's checkpoints expect them. Activations (and their
gradients) are in the compute dtype (fp32 parity mode or bf16); weight / bias / norm-parameter
gradients are fp32.

Backward formulations (reference modules whose autograd they replace are cited per op):
  conv   dX = conv(dY, W flipped/transposed, pad k-1-p) on the forward implicit-GEMM kernel (stride 2:
         dY zero-inserted; nearest-up input: 2x2 sum of the result); dW = split-K GEMM dY^T . im2col(X);
         db / d(timestep emb) = column sums of dY
  norms  GroupNorm(+SiLU) / LayerNorm closed-form backward with the saved / recomputed statistics
  attn   materialised softmax(QK^T s) V: dP = dO V^T, dS = P (dP - rowsum(P dP)) s, dQ = dS K,
         dK = dS^T Q, dV = P^T dO, all strided batched MFMA GEMMs over (image, head)
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Optional

import torch

from . import _lib, ops
from ._lib import GemmDesc, call

NONE, LEAKY, GELU, SILU = ops.NONE, ops.LEAKY, ops.GELU, ops.SILU


def _dt(t: torch.Tensor) -> int:
    return ops.dt_code(t)


def _sp() -> int:
    return ops.stream_ptr()


def gemm(a, a_off: int, a_sm: int, a_sk: int, b, b_off: int, b_sk: int, b_sn: int, c, c_off: int, c_sm: int, *,
         m: int, n: int, k: int, batch: int = 1, nb2: int = 1, a_bs=(0, 0), b_bs=(0, 0), c_bs=(0, 0),
         ksplit: int = 0, alpha: float = 1.0, beta: float = 0.0, rsum=None, rsum_bs: int = 0) -> None:
    """rdeic_gemm_strided on tensors: element offsets / strides in elements of each tensor. rsum: fp32
    tensor receiving A's row sums per batch plane z1 (plane stride rsum_bs)."""
    if a.dtype != b.dtype:
        raise TypeError("gemm operands must share a dtype")
    if c.dtype not in (torch.float32, a.dtype):
        raise TypeError("gemm output must be fp32 or the input dtype")
    d = GemmDesc()
    ea, eb, ec = a.element_size(), b.element_size(), c.element_size()
    d.a, d.a_bs1, d.a_bs2, d.a_sm, d.a_sk = a.data_ptr() + a_off * ea, a_bs[0], a_bs[1], a_sm, a_sk
    d.b, d.b_bs1, d.b_bs2, d.b_sk, d.b_sn = b.data_ptr() + b_off * eb, b_bs[0], b_bs[1], b_sk, b_sn
    d.c, d.c_bs1, d.c_bs2, d.c_sm = c.data_ptr() + c_off * ec, c_bs[0], c_bs[1], c_sm
    d.batch, d.nb2, d.m, d.n, d.k, d.ksplit = batch, nb2, m, n, k, ksplit
    d.dtype = _dt(a)
    d.c_f32 = int(c.dtype == torch.float32 and a.dtype != torch.float32)
    d.alpha, d.beta = alpha, beta
    if rsum is not None:
        if rsum.dtype != torch.float32:
            raise TypeError("row sums are fp32")
        d.rsum, d.rsum_bs = rsum.data_ptr(), rsum_bs
    call("rdeic_gemm_strided", C.byref(d), _sp())


def col_sum(x2d_ptr_tensor: torch.Tensor, rows: int, c: int, ld: int, groups: int = 1, out=None,
            accumulate: bool = False) -> torch.Tensor:
    """[groups, c] fp32 sums over equal row groups of a [rows][ld] view (bias / emb gradients)."""
    if out is None:
        out = torch.empty((groups, c), dtype=torch.float32, device=x2d_ptr_tensor.device)
    nws = int(_lib.load().rdeic_col_sum_ws_floats(rows, c, groups))
    ws = torch.empty(max(nws, 1), dtype=torch.float32, device=x2d_ptr_tensor.device)
    call("rdeic_col_sum", x2d_ptr_tensor.data_ptr(), rows, c, ld, groups, out.data_ptr(), int(accumulate),
         ws.data_ptr(), nws, _dt(x2d_ptr_tensor), _sp())
    return out


def _rows_view(t: torch.Tensor):
    """(rows, c, ld) of an NHWC activation or a [rows, c] token tensor (channel-contiguous)."""
    if t.dim() == 4:
        ld = ops.pix_ld(t)
        return t.shape[0] * t.shape[1] * t.shape[2], t.shape[3], ld
    if t.dim() == 2 and t.stride(1) == 1:
        return t.shape[0], t.shape[1], t.stride(0)
    raise ValueError(f"expected NHWC or [rows, c] with contiguous channels, got {tuple(t.shape)} {t.stride()}")


# ---------------------------------------------------------------------------------------- conv / linear
@dataclass(frozen=True)
class ConvCfg:
    kh: int
    kw: int
    stride: int = 1
    pad: int = 0
    up2: bool = False
    pixel_shuffle: bool = False
    act: int = NONE
    slope: float = 0.0
    out_f32: bool = False
    key: Optional[str] = None  # cache key of a frozen layer's packed weights (see TrainOps)


class PackCache:
    """Packed forward / dgrad weights of FROZEN layers (packed once); trainable layers repack per step."""

    def __init__(self):
        self.fwd, self.dgrad = {}, {}

    def clear(self):
        self.fwd.clear()
        self.dgrad.clear()


PACKS = PackCache()


class StepPacks:
    """Packed forward / input-gradient weights of the TRAINABLE layers, refreshed once per step by a
    single rdeic_pack_batch launch (in place of one pack launch per layer and use). A layer is
    registered the first time a step packs it (packed alone then); from the next step on, refresh()
    repacks every registered layer after the optimizer update, before the forward. Used only while
    active (FineTuner's step), since the packs are valid only between refresh() and the update."""

    def __init__(self):
        self.entries = {}          # (id(weight), dtype, mode) -> (packed tensor, wld)
        self.jobs = []             # (weight, packed, cout, cin, kh, kw, wld, mode)
        self.table = None          # device job table (rdeic_pack_job[])
        self.total = 0
        self.dtype = None
        self.on = False

    def clear(self):
        self.__init__()

    def active(self):
        sp = self

        class _Ctx:
            def __enter__(self_):
                self_.prev, sp.on = sp.on, True

            def __exit__(self_, *exc):
                sp.on = self_.prev
        return _Ctx()

    def lookup(self, w, dtype, mode):
        if not self.on:
            return None
        e = self.entries.get((id(w), dtype, mode))
        if e is not None and self.table is not None and e[2]:
            return e[0], e[1]
        return None

    def register(self, w, dtype, mode, packed, wld, cout, cin, kh, kw):
        if not self.on or (self.dtype is not None and dtype != self.dtype):
            return
        key = (id(w), dtype, mode)
        if key in self.entries:
            return
        self.dtype = dtype
        self.entries[key] = (packed, wld, False)  # usable from the next refresh on
        self.jobs.append((w, packed, cout, cin, kh, kw, wld, mode))
        self.table = None

    def refresh(self):
        """Repack every registered layer (one launch). Builds the device job table when layers were
        added since the last refresh (host->device copy: call outside graph capture then)."""
        if not self.jobs:
            return
        if self.table is None:
            rows, start, self.row_floats = [], 0, 1
            for w, packed, cout, cin, kh, kw, wld, mode in self.jobs:
                self.row_floats = max(self.row_floats, kh * kw * (cin if mode == 0 else cout))
                if self.row_floats > 36864:
                    raise ValueError("rdeic_pack_batch: a packed row's sources exceed the LDS staging limit")
                rows.append((w.data_ptr(), packed.data_ptr(), start, cout | (cin << 32), kh | (kw << 32),
                             wld | (mode << 32)))
                start += packed.shape[0]  # output rows
            self.total = start
            self.table = torch.tensor(rows, dtype=torch.int64).to(self.jobs[0][1].device)
            for k, (packed, wld, _) in list(self.entries.items()):
                self.entries[k] = (packed, wld, True)
        call("rdeic_pack_batch", self.table.data_ptr(), len(self.jobs), self.total, self.row_floats,
             int(self.dtype == torch.bfloat16), _sp())


STEP_PACKS = StepPacks()


def _pack_fwd(weight: torch.Tensor, bias, cfg: ConvCfg, dtype, frozen: bool) -> ops.ConvParams:
    key = (cfg.key, cfg.stride, cfg.pad, dtype)
    if frozen and cfg.key is not None and key in PACKS.fwd:
        return PACKS.fwd[key]
    if not frozen:
        hit = STEP_PACKS.lookup(weight, dtype, 0)
        if hit is not None:
            w4 = weight if weight.dim() == 4 else weight[:, :, None, None]
            cout, cin, kh, kw = w4.shape
            b = None if bias is None else bias.detach()
            return ops.ConvParams(hit[0], hit[1], b, cout, cin, kh, kw, cfg.stride, cfg.pad)
    p = ops.ConvParams.pack(weight.detach(), None if bias is None else bias.detach(), stride=cfg.stride,
                            pad=cfg.pad, dtype=dtype)
    if frozen and cfg.key is not None:
        PACKS.fwd[key] = p
    elif not frozen:
        STEP_PACKS.register(weight, dtype, 0, p.weight, p.wld, p.cout, p.cin, p.kh, p.kw)
    return p


def _pack_dgrad(weight: torch.Tensor, dtype, frozen: bool, key) -> tuple:
    ck = (key, dtype)
    if frozen and key is not None and ck in PACKS.dgrad:
        return PACKS.dgrad[ck]
    if not frozen:
        hit = STEP_PACKS.lookup(weight, dtype, 1)
        if hit is not None:
            return hit
    w = weight.detach()
    if w.dim() == 2:
        w = w[:, :, None, None]
    w = w.contiguous()
    cout, cin, kh, kw = w.shape
    wld = -(-(kh * kw * cout) // 64) * 64
    packed = torch.empty((cin, wld), dtype=dtype, device=w.device)
    call("rdeic_pack_conv_weight_dgrad", w.data_ptr(), cout, cin, kh, kw, packed.data_ptr(), wld,
         int(dtype == torch.bfloat16), _sp())
    r = (packed, wld)
    if frozen and key is not None:
        PACKS.dgrad[ck] = r
    elif not frozen:
        STEP_PACKS.register(weight, dtype, 1, packed, wld, cout, cin, kh, kw)
    return r


def conv_dgrad(dz: torch.Tensor, weight: torch.Tensor, cfg: ConvCfg, in_hw, frozen: bool) -> torch.Tensor:
    """Input gradient of a conv whose output gradient (after act / unshuffle) is dz [n, ho, wo, cout]."""
    cout, cin = weight.shape[0], weight.shape[1]
    packed, wld = _pack_dgrad(weight, dz.dtype, frozen, cfg.key)
    p = ops.ConvParams(packed, wld, None, cin, cout, cfg.kh, cfg.kw, 1, cfg.kh - 1 - cfg.pad)
    n = dz.shape[0]
    h, w = in_hw
    hi, wi = (2 * h, 2 * w) if cfg.up2 else (h, w)
    src = dz
    if cfg.stride == 2:
        if hi != 2 * dz.shape[1] or wi != 2 * dz.shape[2]:
            raise ValueError("stride-2 conv backward needs an even input size")
        src = torch.empty((n, hi, wi, cout), dtype=dz.dtype, device=dz.device)
        call("rdeic_zero_insert2", dz.data_ptr(), n, dz.shape[1], dz.shape[2], cout, ops.pix_ld(dz), src.data_ptr(),
             cout, _dt(dz), _sp())
    elif cfg.stride != 1:
        raise ValueError("conv backward supports stride 1 and 2")
    d_in = ops.conv2d(src, p, out_hw=(hi, wi))
    if cfg.up2:
        dx = torch.empty((n, h, w, cin), dtype=dz.dtype, device=dz.device)
        call("rdeic_sum_pool2", d_in.data_ptr(), n, h, w, cin, cin, dx.data_ptr(), cin, _dt(dz), _sp())
        return dx
    return d_in


# Direct gradients: a trainable parameter may carry `_rdeic_gview` (its fp32 gradient view, e.g. a
# slice of FineTuner's flat buffer) and `_rdeic_notify` (called once its gradient is complete, e.g.
# the DDP bucket counter). The conv / linear backward then accumulates the weight and bias gradients
# straight into the view (the finalize kernels' accumulate mode) and returns None for them, so
# autograd runs no AccumulateGrad add per parameter. The sums equal AccumulateGrad's (0 + g = g).
# A parameter used by several layers (the checkerboard entropy nets run on the anchor and the
# non-anchor half) is notified after its last use's gradient: the forward counts the uses that
# will run a backward, each backward contribution counts one down.
def direct_grad_view(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else getattr(t, "_rdeic_gview", None)


def count_direct_use(t: Optional[torch.Tensor], needs_grad: bool) -> Optional[torch.Tensor]:
    """Forward side (needs_grad: the Function's ctx.needs_input_grad entry for t — grad mode itself
    is off inside Function.forward): the parameter if its gradient will go to its direct view."""
    if direct_grad_view(t) is None or not needs_grad:
        return None
    t._rdeic_uses = getattr(t, "_rdeic_uses", 0) + 1
    t._rdeic_direct = True  # autograd still runs the leaf's AccumulateGrad (on no gradient): hooks skip it
    return t


def notify_grad(t: torch.Tensor) -> None:
    t._rdeic_uses -= 1
    if t._rdeic_uses == 0:
        fn = getattr(t, "_rdeic_notify", None)
        if fn is not None:
            fn(t)


def conv_wgrad(x: torch.Tensor, dz: torch.Tensor, cfg: ConvCfg, cout: int, cin: int, out=None,
               accumulate: bool = False, db: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 [cout, cin, kh, kw] = dz^T . im2col(x) (split-K over pixels, fixed-order reduction)."""
    n, ho, wo, _ = dz.shape
    P = n * ho * wo
    K = cfg.kh * cfg.kw * cin
    ldz = ops.pix_ld(dz)
    if cfg.kh == 1 and cfg.kw == 1 and cfg.stride == 1 and not cfg.up2 and cfg.pad == 0:
        cols, b_sk = x, ops.pix_ld(x)
    else:
        cols = torch.empty((P, K), dtype=x.dtype, device=x.device)
        call("rdeic_im2col", x.data_ptr(), x.shape[0], x.shape[1], x.shape[2], cin, ops.pix_ld(x), cfg.kh, cfg.kw,
             cfg.stride, cfg.pad, cfg.pad, ho, wo, int(cfg.up2), cols.data_ptr(), K, _dt(x), _sp())
        b_sk = K
    tiles = -(-cout // 64) * -(-K // 64)
    splits = max(1, min(-(-1024 // tiles), -(-P // 256), 64))
    ks = -(-P // splits)
    ks = -(-ks // 32) * 32
    splits = -(-P // ks)
    part = torch.empty((splits, cout, K), dtype=torch.float32, device=x.device)
    # db: the bias gradient (column sums of dz) as the GEMM's row sums of A = dz^T, same accumulate mode
    rpart = torch.empty((splits, cout), dtype=torch.float32, device=x.device) if db is not None else None
    gemm(dz, 0, 1, ldz, cols, 0, b_sk, 1, part, 0, K, m=cout, n=K, k=P, batch=splits, c_bs=(cout * K, 0), ksplit=ks,
         rsum=rpart, rsum_bs=cout)
    if out is None:
        out = torch.empty((cout, cin, cfg.kh, cfg.kw), dtype=torch.float32, device=x.device)
    call("rdeic_wgrad_finalize", part.data_ptr(), splits, cout, cin, cfg.kh, cfg.kw, out.data_ptr(), int(accumulate),
         None if db is None else rpart.data_ptr(), None if db is None else db.data_ptr(), _sp())
    return out


def _conv_forward(x, weight, bias, emb, res, cfg: ConvCfg):
    """(out, z): z = conv(x) + bias + emb (pre-activation, kept only when cfg.act != NONE)."""
    frozen = not weight.requires_grad
    p = _pack_fwd(weight, bias, cfg, x.dtype, frozen)
    if p.cin != x.shape[3]:
        raise ValueError(f"conv expects {p.cin} input channels, got {x.shape[3]}")
    fused_res = res if cfg.act == NONE else None
    z = ops.conv2d(x, p, up2=cfg.up2, emb=emb, res=fused_res, out_f32=cfg.out_f32, pixel_shuffle=cfg.pixel_shuffle)
    if cfg.act == NONE:
        return z, None
    rows, c, ldz = _rows_view(z)
    out = torch.empty_like(z)
    r_ld = 0
    if res is not None:
        if res.shape != z.shape or res.dtype != z.dtype:
            raise ValueError("residual must match the conv output")
        r_ld = _rows_view(res)[2]
    call("rdeic_act_fwd", z.data_ptr(), rows, c, ldz, None if res is None else res.data_ptr(), r_ld, cfg.act,
         float(cfg.slope), out.data_ptr(), c, _dt(z), _sp())
    return out, z


def _conv_backward(x, weight, z, dout, cfg: ConvCfg, in_hw, need_x, need_w, need_b, need_emb, bias=None):
    """(dx, dw, db, demb) of _conv_forward given the output gradient (dres = dout). dw / db are None
    when they went straight into the parameters' direct gradient views (direct_grad_view)."""
    dz = dout
    if cfg.act != NONE:
        rows, c, ldz = _rows_view(z)
        dz = torch.empty_like(z)
        call("rdeic_act_bwd", dout.data_ptr(), _rows_view(dout)[2], z.data_ptr(), ldz, rows, c, cfg.act,
             float(cfg.slope), dz.data_ptr(), c, _dt(z), _sp())
    if cfg.pixel_shuffle:
        n, H2, W2, c = dz.shape
        u = torch.empty((n, H2 // 2, W2 // 2, 4 * c), dtype=dz.dtype, device=dz.device)
        call("rdeic_pixel_unshuffle2", dz.data_ptr(), n, H2 // 2, W2 // 2, c, ops.pix_ld(dz), u.data_ptr(), 4 * c,
             _dt(dz), _sp())
        dz = u
    cout, cin = weight.shape[0], weight.shape[1]
    if dz.dtype != x.dtype:  # fp32 output of a bf16 conv: gradients flow back in the compute dtype
        dz = ops.cast(dz.contiguous(), x.dtype)
    elif ops.pix_ld(dz) != cout:
        dz = dz.contiguous()
    n, ho, wo, _ = dz.shape
    dx = dw = db = demb = None
    if need_x:
        dx = conv_dgrad(dz, weight, cfg, in_hw, frozen=not weight.requires_grad)
    gvw = direct_grad_view(weight) if need_w and getattr(weight, "_rdeic_uses", 0) > 0 else None
    gvb = direct_grad_view(bias) if need_b else None  # bias is passed only when counted in the forward
    fuse_b = gvw is not None and gvb is not None  # bias gradient from the weight-gradient GEMM's row sums
    if need_w:
        if gvw is not None:
            conv_wgrad(x, dz, cfg, cout, cin, out=gvw, accumulate=True, db=gvb if fuse_b else None)
            notify_grad(weight)
        else:
            dw = conv_wgrad(x, dz, cfg, cout, cin).view(weight.shape)
    if need_b:
        if fuse_b:
            notify_grad(bias)
        elif gvb is not None:
            col_sum(dz, n * ho * wo, cout, cout, out=gvb.view(1, cout), accumulate=True)
            notify_grad(bias)
        else:
            db = col_sum(dz, n * ho * wo, cout, cout).view(cout)
    if need_emb:
        demb = col_sum(dz, n * ho * wo, cout, cout, groups=n)
    return dx, dw, db, demb


class Conv2dFn(torch.autograd.Function):
    """out = act(conv(x) + bias + emb[img]) + res   (NHWC; PixelShuffle(2) after the conv when set)."""

    @staticmethod
    def forward(ctx, x, weight, bias, emb, res, cfg: ConvCfg):
        out, z = _conv_forward(x, weight, bias, emb, res, cfg)
        ctx.cfg = cfg
        ctx.flags = (emb is not None, res is not None, bias is not None)
        ctx.in_hw = (x.shape[1], x.shape[2])
        count_direct_use(weight, ctx.needs_input_grad[1])
        ctx.bias = count_direct_use(bias, ctx.needs_input_grad[2])  # a leaf parameter
        ctx.splitk = ops.splitk_state()  # the backward runs on autograd's engine thread (ops.splitk_as)
        ctx.save_for_backward(x, weight, z)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, weight, z = ctx.saved_tensors
        has_emb, has_res, has_bias = ctx.flags
        dout = dout.contiguous()
        nig = ctx.needs_input_grad
        with ops.splitk_as(ctx.splitk):
            dx, dw, db, demb = _conv_backward(x, weight, z, dout, ctx.cfg, ctx.in_hw, nig[0], nig[1],
                                              has_bias and nig[2], has_emb and nig[3], bias=ctx.bias)
        return dx, dw, db, demb, (dout if has_res else None), None


def conv2d(x, weight, bias=None, *, emb=None, res=None, cfg: ConvCfg):
    return Conv2dFn.apply(x, weight, bias, emb, res, cfg)


def _tok4(t: torch.Tensor) -> torch.Tensor:
    rows, c = t.shape
    return t.as_strided((1, rows, 1, c), (rows * t.stride(0), t.stride(0), t.stride(0), 1))


class LinearFn(torch.autograd.Function):
    """Token-wise nn.Linear over [rows, cin] (row stride allowed) on the 1x1-conv kernels;
    out = x W^T + b (+ res)."""

    @staticmethod
    def forward(ctx, x, weight, bias, res, cfg: ConvCfg):
        rows = x.shape[0]
        out, _ = _conv_forward(_tok4(x), weight, bias, None, None if res is None else _tok4(res), cfg)
        ctx.cfg = cfg
        ctx.flags = (res is not None, bias is not None)
        count_direct_use(weight, ctx.needs_input_grad[1])
        ctx.bias = count_direct_use(bias, ctx.needs_input_grad[2])
        ctx.splitk = ops.splitk_state()
        ctx.save_for_backward(x, weight)
        return out.view(rows, weight.shape[0])

    @staticmethod
    def backward(ctx, dout):
        x, weight = ctx.saved_tensors
        has_res, has_bias = ctx.flags
        dout = dout.contiguous()
        rows = x.shape[0]
        nig = ctx.needs_input_grad
        with ops.splitk_as(ctx.splitk):
            dx, dw, db, _ = _conv_backward(_tok4(x), weight, None, _tok4(dout), ctx.cfg, (rows, 1), nig[0], nig[1],
                                           has_bias and nig[2], False, bias=ctx.bias)
        if dx is not None:
            dx = dx.view(rows, weight.shape[1])
        return dx, dw, db, (dout if has_res else None), None


def linear(x2d: torch.Tensor, weight, bias=None, *, res=None, key=None, out_f32=False):
    return LinearFn.apply(x2d, weight, bias, res, ConvCfg(1, 1, key=key, out_f32=out_f32))


class CastFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src = x.dtype
        return ops.cast(x, dtype)

    @staticmethod
    def backward(ctx, g):
        return ops.cast(g.contiguous(), ctx.src), None


def cast(x: torch.Tensor, dtype) -> torch.Tensor:
    return x if x.dtype == dtype else CastFn.apply(x, dtype)


class ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, act: int, slope: float):
        z = z.contiguous()
        out = torch.empty_like(z)
        c = z.shape[-1]
        call("rdeic_act_fwd", z.data_ptr(), z.numel() // c, c, c, None, 0, act, float(slope), out.data_ptr(), c,
             _dt(z), _sp())
        ctx.act, ctx.slope = act, slope
        ctx.save_for_backward(z)
        return out

    @staticmethod
    def backward(ctx, g):
        (z,) = ctx.saved_tensors
        g = g.contiguous()
        dz = torch.empty_like(z)
        c = z.shape[-1]
        call("rdeic_act_bwd", g.data_ptr(), c, z.data_ptr(), c, z.numel() // c, c, ctx.act, float(ctx.slope),
             dz.data_ptr(), c, _dt(z), _sp())
        return dz, None, None


def act(z, kind: int, slope: float = 0.0):
    return ActFn.apply(z, kind, slope)


# ------------------------------------------------------------------------------------------- norms
def _count_direct_pair(ctx, gamma, beta) -> bool:
    """A norm's (gamma, beta): both go to their direct gradient views (the backward kernel's accumulate mode,
    no AccumulateGrad add per parameter) when both have one and both need a gradient; else neither does."""
    nig = ctx.needs_input_grad
    if nig[1] and nig[2] and direct_grad_view(gamma) is not None and direct_grad_view(beta) is not None:
        count_direct_use(gamma, True)
        count_direct_use(beta, True)
        return True
    return False


def _param_grad_targets(ctx, gamma, beta, c: int, device):
    """(dgamma, dbeta, accumulate) for a norm backward: the direct views (accumulate) or fresh tensors."""
    if ctx.direct:
        return direct_grad_view(gamma), direct_grad_view(beta), 1
    if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
        return (torch.empty(c, dtype=torch.float32, device=device), torch.empty(c, dtype=torch.float32, device=device), 0)
    return None, None, 0


def _res_grad(dxa, x):
    """(pointer, row stride) of a passthrough alias's gradient (None: no gradient reached the alias)."""
    if dxa is None:
        return None, 0
    if dxa.dtype != x.dtype or dxa.shape != x.shape:
        raise ValueError("residual gradient must match the norm input")
    dxa = dxa.contiguous()
    return dxa.data_ptr(), dxa.shape[-1]


class GroupNormFn(torch.autograd.Function):
    """y = silu?(GroupNorm(x)) over NHWC x (GroupNorm32 / GroupNorm_leq32 / Normalize + SiLU)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, groups: int, eps: float, silu: bool, passthrough: bool = False):
        n, h, w, c = x.shape
        hw = h * w
        ld = ops.pix_ld(x)
        mr = torch.empty((n, groups, 2), dtype=torch.float32, device=x.device)
        ab = torch.empty((n, c, 2), dtype=torch.float32, device=x.device)
        ws = torch.empty(int(_lib.load().rdeic_gn_train_ws_doubles(n, hw, c)), dtype=torch.float64, device=x.device)
        call("rdeic_gn_train_fwd", x.data_ptr(), ld, n, hw, c, groups, float(eps), gamma.data_ptr(), beta.data_ptr(),
             mr.data_ptr(), ab.data_ptr(), ws.data_ptr(), _dt(x), _sp())
        y = ops.group_norm_apply(x, ab, silu)
        ctx.groups, ctx.silu = groups, silu
        ctx.direct = _count_direct_pair(ctx, gamma, beta)
        ctx.save_for_backward(x, gamma, beta, mr)
        if passthrough:  # (y, x): x's other consumer takes the alias, its gradient comes back here (_res_grad)
            ctx.set_materialize_grads(False)
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dxa=None):
        x, gamma, beta, mr = ctx.saved_tensors
        dy = dy.contiguous()
        n, h, w, c = x.shape
        hw = h * w
        dx = torch.empty((n, h, w, c), dtype=x.dtype, device=x.device)
        dg, dbt, acc = _param_grad_targets(ctx, gamma, beta, c, x.device)
        ws = torch.empty(int(_lib.load().rdeic_gn_train_ws_doubles(n, hw, c)), dtype=torch.float64, device=x.device)
        coef = torch.empty((n, ctx.groups, 2), dtype=torch.float32, device=x.device)
        dres, ldr = _res_grad(dxa, x)
        call("rdeic_gn_train_bwd_res", x.data_ptr(), ops.pix_ld(x), dy.data_ptr(), c, n, hw, c, ctx.groups,
             mr.data_ptr(), gamma.data_ptr(), beta.data_ptr(), int(ctx.silu), dres, ldr, dx.data_ptr(), c,
             None if dg is None else dg.data_ptr(), None if dbt is None else dbt.data_ptr(), acc, ws.data_ptr(),
             coef.data_ptr(), _dt(x), _sp())
        if ctx.direct:
            notify_grad(gamma)
            notify_grad(beta)
            return dx, None, None, None, None, None, None
        return dx, dg, dbt, None, None, None, None


def group_norm(x, gamma, beta, groups: int, eps: float, silu: bool, passthrough: bool = False):
    """passthrough: also return an alias of x for x's second consumer (a residual / skip path); that consumer's
    gradient is then added inside this norm's backward kernel instead of by an autograd add launch."""
    return GroupNormFn.apply(x, gamma, beta, groups, eps, silu, passthrough)


class LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps: float, passthrough: bool = False):
        rows, c = x.shape
        y = torch.empty((rows, c), dtype=x.dtype, device=x.device)
        call("rdeic_layernorm", x.data_ptr(), rows, c, x.stride(0), gamma.data_ptr(), beta.data_ptr(), float(eps),
             y.data_ptr(), c, _dt(x), _sp())
        ctx.eps = eps
        ctx.direct = _count_direct_pair(ctx, gamma, beta)
        ctx.save_for_backward(x, gamma, beta)
        if passthrough:
            ctx.set_materialize_grads(False)
            return y, x.view_as(x)
        return y

    @staticmethod
    def backward(ctx, dy, dxa=None):
        x, gamma, beta = ctx.saved_tensors
        dy = dy.contiguous()
        rows, c = x.shape
        dx = torch.empty((rows, c), dtype=x.dtype, device=x.device)
        dg, db, acc = _param_grad_targets(ctx, gamma, beta, c, x.device)
        ws = None
        nws = 0
        if dg is not None:
            nws = int(_lib.load().rdeic_layernorm_bwd_ws_floats(rows, c))
            ws = torch.empty(nws, dtype=torch.float32, device=x.device)
        dres, ldr = _res_grad(dxa, x)
        call("rdeic_layernorm_bwd_res", x.data_ptr(), x.stride(0), rows, c, gamma.data_ptr(), float(ctx.eps),
             dy.data_ptr(), c, dres, ldr, dx.data_ptr(), c, None if dg is None else dg.data_ptr(),
             None if db is None else db.data_ptr(), acc, None if ws is None else ws.data_ptr(), nws, _dt(x), _sp())
        if ctx.direct:
            notify_grad(gamma)
            notify_grad(beta)
            return dx, None, None, None, None
        return dx, dg, db, None, None


def layer_norm(x, gamma, beta, eps: float = 1e-5, passthrough: bool = False):
    """passthrough: as group_norm's (the transformer's residual around each LayerNorm)."""
    return LayerNormFn.apply(x, gamma, beta, eps, passthrough)


# --------------------------------------------------------------------------------------- attention
def _heads_gemm(a, a_sm: int, a_sk: int, a_bs, b, b_sk: int, b_sn: int, b_bs, *, m: int, n: int, k: int, batch: int,
                heads: int, dt, dev) -> torch.Tensor:
    """Per (image, head) C = A B into a [batch * m, heads * n] token tensor (attention's P V, dS K,
    dS^T Q, P^T dO). These have few output tiles (n = head dim) and a long k: at batch 1 (the
    fine-tune step) k is split so the grid fills the chip, then the planes are summed in order."""
    out = torch.empty((batch * m, heads * n), dtype=dt, device=dev)
    tiles = -(-m // 64) * -(-n // 64) * batch * heads
    splits = max(1, min(-(-1024 // tiles), k // 256)) if (batch == 1 and tiles < 512 and k >= 512) else 1
    if splits == 1:
        gemm(a, 0, a_sm, a_sk, b, 0, b_sk, b_sn, out, 0, heads * n, m=m, n=n, k=k, batch=batch * heads, nb2=heads,
             a_bs=a_bs, b_bs=b_bs, c_bs=(m * heads * n, n))
        return out
    ks = -(-k // splits)
    ks = -(-ks // 32) * 32
    ns = -(-k // ks)
    plane = m * heads * n
    part = torch.empty((ns, plane), dtype=torch.float32, device=dev)
    gemm(a, 0, a_sm, a_sk, b, 0, b_sk, b_sn, part, 0, heads * n, m=m, n=n, k=k, batch=ns * heads, nb2=heads,
         a_bs=(0, a_bs[1]), b_bs=(0, b_bs[1]), c_bs=(plane, n), ksplit=ks)
    if dt == torch.float32:
        col_sum(part, ns, plane, plane, out=out.view(1, plane))
        return out
    tot = col_sum(part, ns, plane, plane)
    call("rdeic_cast", tot.data_ptr(), ops.dt_code(tot), out.data_ptr(), ops.dt_code(out), plane, _sp())
    return out


class AttentionFn(torch.autograd.Function):
    """softmax(Q K^T * scale) V per (image, head) over 'b n (h d)' token tensors (CrossAttention.forward,
    attention.py:171-203), materialised: P is kept for the backward."""

    @staticmethod
    def forward(ctx, q, k, v, batch: int, heads: int, scale: float):
        Lq = q.shape[0] // batch
        Lk = k.shape[0] // batch
        dh = q.shape[1] // heads
        dev, dt = q.device, q.dtype
        s = torch.empty((batch, heads, Lq, Lk), dtype=torch.float32, device=dev)
        ldq, ldk, ldv = q.stride(0), k.stride(0), v.stride(0)
        gemm(q, 0, ldq, 1, k, 0, 1, ldk, s, 0, Lk, m=Lq, n=Lk, k=dh, batch=batch * heads, nb2=heads,
             a_bs=(Lq * ldq, dh), b_bs=(Lk * ldk, dh), c_bs=(heads * Lq * Lk, Lq * Lk))
        p = torch.empty((batch, heads, Lq, Lk), dtype=dt, device=dev)
        call("rdeic_softmax_rows", s.data_ptr(), batch * heads * Lq, Lk, float(scale), p.data_ptr(), _dt(q), _sp())
        del s
        o = _heads_gemm(p, Lk, 1, (heads * Lq * Lk, Lq * Lk), v, ldv, 1, (Lk * ldv, dh), m=Lq, n=dh, k=Lk,
                        batch=batch, heads=heads, dt=dt, dev=dev)
        ctx.dims = (batch, heads, Lq, Lk, dh, scale)
        ctx.save_for_backward(q, k, v, p)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, p = ctx.saved_tensors
        batch, heads, Lq, Lk, dh, scale = ctx.dims
        do = do.contiguous()
        dev, dt = q.device, q.dtype
        ldq, ldk, ldv, ldo = q.stride(0), k.stride(0), v.stride(0), do.stride(0)
        nb = batch * heads
        dp = torch.empty((batch, heads, Lq, Lk), dtype=torch.float32, device=dev)
        gemm(do, 0, ldo, 1, v, 0, 1, ldv, dp, 0, Lk, m=Lq, n=Lk, k=dh, batch=nb, nb2=heads,
             a_bs=(Lq * ldo, dh), b_bs=(Lk * ldv, dh), c_bs=(heads * Lq * Lk, Lq * Lk))
        ds = torch.empty((batch, heads, Lq, Lk), dtype=dt, device=dev)
        call("rdeic_softmax_bwd_rows", p.data_ptr(), dp.data_ptr(), nb * Lq, Lk, float(scale), ds.data_ptr(), _dt(q),
             _sp())
        del dp
        pl = (heads * Lq * Lk, Lq * Lk)
        dq = dk = dv = None
        if ctx.needs_input_grad[0]:
            dq = _heads_gemm(ds, Lk, 1, pl, k, ldk, 1, (Lk * ldk, dh), m=Lq, n=dh, k=Lk, batch=batch, heads=heads,
                             dt=dt, dev=dev)
        if ctx.needs_input_grad[1]:
            dk = _heads_gemm(ds, 1, Lk, pl, q, ldq, 1, (Lq * ldq, dh), m=Lk, n=dh, k=Lq, batch=batch, heads=heads,
                             dt=dt, dev=dev)
        if ctx.needs_input_grad[2]:
            dv = _heads_gemm(p, 1, Lk, pl, do, ldo, 1, (Lq * ldo, dh), m=Lk, n=dh, k=Lq, batch=batch, heads=heads,
                             dt=dt, dev=dev)
        return dq, dk, dv, None, None, None


def attention(q, k, v, batch: int, heads: int, scale: float):
    return AttentionFn.apply(q, k, v, batch, heads, scale)


class GegluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        rows, c2 = x.shape
        c = c2 // 2
        out = torch.empty((rows, c), dtype=x.dtype, device=x.device)
        call("rdeic_geglu", x.data_ptr(), rows, c, x.stride(0), out.data_ptr(), c, _dt(x), _sp())
        ctx.save_for_backward(x)
        return out

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous()
        rows, c2 = x.shape
        dx = torch.empty((rows, c2), dtype=x.dtype, device=x.device)
        call("rdeic_geglu_bwd", x.data_ptr(), x.stride(0), rows, c2 // 2, dy.data_ptr(), c2 // 2, dx.data_ptr(), c2,
             _dt(x), _sp())
        return dx


def geglu(x):
    return GegluFn.apply(x)


# ------------------------------------------------------------------------- checkerboard entropy model
class CkbdMaskFn(torch.autograd.Function):
    """x at anchor (which=1) / non-anchor (which=0) positions, 0 elsewhere (utils/ckbd.py:33-45)."""

    @staticmethod
    def forward(ctx, x, which: int):
        n, h, w, c = x.shape
        out = torch.empty((n, h, w, c), dtype=x.dtype, device=x.device)
        call("rdeic_ckbd_mask", x.data_ptr(), ops.pix_ld(x), n, h, w, c, which, out.data_ptr(), c, _dt(x), _sp())
        ctx.which = which
        return out

    @staticmethod
    def backward(ctx, g):
        return CkbdMaskFn.apply(g.contiguous(), ctx.which), None


class CkbdAnchorFn(torch.autograd.Function):
    """slice_anchor_hat = quantize_ste(ckbd_anchor(y) - ckbd_anchor(mu_a)) + ckbd_anchor(mu_a)
    (compression.py:86-89): value round(y - mu) + mu at anchors; gradient to y only (STE), none to mu."""

    @staticmethod
    def forward(ctx, y, pa):
        n, h, w, c = y.shape
        out = torch.empty((n, h, w, c), dtype=y.dtype, device=y.device)
        call("rdeic_ckbd_train_anchor", y.data_ptr(), ops.pix_ld(y), pa.data_ptr(), ops.pix_ld(pa), n, h, w, c,
             out.data_ptr(), c, _dt(y), _sp())
        return out

    @staticmethod
    def backward(ctx, g):
        return CkbdMaskFn.apply(g.contiguous(), 1), None


class CkbdLikFn(torch.autograd.Function):
    """One slice's GaussianConditional likelihoods (noise mode -> S = sum ln lik, dequantize mode ->
    qS, no gradient) and the non-anchor half of y_hat (quantize_ste), compression.py:94-106."""

    @staticmethod
    def forward(ctx, y, pa, pn, noise):
        n, h, w, c = y.shape
        non = torch.empty((n, h, w, c), dtype=y.dtype, device=y.device)
        nws = int(_lib.load().rdeic_ckbd_train_ws_doubles(n, h, w, c))
        ws = torch.empty(nws, dtype=torch.float64, device=y.device)
        out2 = torch.empty(2, dtype=torch.float32, device=y.device)
        call("rdeic_ckbd_train_lik", y.data_ptr(), ops.pix_ld(y), pa.data_ptr(), ops.pix_ld(pa), pn.data_ptr(),
             ops.pix_ld(pn), noise.data_ptr(), n, h, w, c, non.data_ptr(), c, ws.data_ptr(), out2.data_ptr(), _dt(y),
             _sp())
        ctx.save_for_backward(y, pa, pn, noise)
        S, qS = out2[0:1].clone(), out2[1:2].clone()
        ctx.mark_non_differentiable(qS)
        return S, qS, non

    @staticmethod
    def backward(ctx, gS, gq, gnon):
        y, pa, pn, noise = ctx.saved_tensors
        n, h, w, c = y.shape
        dy = torch.empty((n, h, w, c), dtype=y.dtype, device=y.device)
        dpa = torch.empty((n, h, w, 2 * c), dtype=y.dtype, device=y.device)
        dpn = torch.empty((n, h, w, 2 * c), dtype=y.dtype, device=y.device)
        gS = gS.to(torch.float32).contiguous()
        gnon = None if gnon is None else gnon.contiguous()
        call("rdeic_ckbd_train_lik_bwd", y.data_ptr(), ops.pix_ld(y), pa.data_ptr(), ops.pix_ld(pa), pn.data_ptr(),
             ops.pix_ld(pn), noise.data_ptr(), n, h, w, c, gS.data_ptr(), None if gnon is None else gnon.data_ptr(), c,
             dy.data_ptr(), c, dpa.data_ptr(), 2 * c, dpn.data_ptr(), 2 * c, _dt(y), _sp())
        return dy, dpa, dpn, None


# ------------------------------------------------------------------------------------ vector quantiser
class VQTrainFn(torch.autograd.Function):
    """VectorQuantiser.forward in training mode (compression_modules.py:228-307): nearest code,
    commitment loss, contrastive loss, EMA usage and dead-code re-initialisation (in place on E and
    embed_prob, like the reference's .data update). Returns (z_q straight-through, emb_loss[1])."""

    @staticmethod
    def forward(ctx, z, E, embed_prob, beta: float, decay: float, temp: float):
        B, hz, wz, D = z.shape
        P = B * hz * wz
        K = E.shape[0]
        dev = z.device
        zf = ops.cast(z.contiguous(), torch.float32).view(P, D)
        Ed = E.detach()
        dot = torch.empty((P, K), dtype=torch.float32, device=dev)
        gemm(zf, 0, D, 1, Ed, 0, 1, D, dot, 0, K, m=P, n=K, k=D)
        zn = torch.empty(P, dtype=torch.float32, device=dev)
        en = torch.empty(K, dtype=torch.float32, device=dev)
        call("rdeic_row_sqnorm", zf.data_ptr(), P, D, D, zn.data_ptr(), 0, _sp())
        call("rdeic_row_sqnorm", Ed.data_ptr(), K, D, D, en.data_ptr(), 0, _sp())
        idx = torch.empty(P, dtype=torch.int32, device=dev)
        call("rdeic_vq_argmin", dot.data_ptr(), zn.data_ptr(), en.data_ptr(), P, K, idx.data_ptr(), _sp())
        zq = torch.empty((P, D), dtype=torch.float32, device=dev)
        call("rdeic_gather_rows", Ed.data_ptr(), D, idx.data_ptr(), P, D, zq.data_ptr(), D, 0, _sp())
        code_out = torch.empty((K, 2), dtype=torch.float32, device=dev)
        dE_unit = torch.empty((K, D), dtype=torch.float32, device=dev)
        loss3 = torch.empty(3, dtype=torch.float32, device=dev)
        call("rdeic_vq_train", dot.data_ptr(), zn.data_ptr(), en.data_ptr(), zf.data_ptr(), idx.data_ptr(), P, K, D,
             Ed.data_ptr(), embed_prob.data_ptr(), float(beta), float(decay), float(temp), code_out.data_ptr(),
             dE_unit.data_ptr(), loss3.data_ptr(), _sp())
        ctx.beta, ctx.shape, ctx.dt = beta, (B, hz, wz, D), z.dtype
        ctx.save_for_backward(zf, zq, dE_unit)
        ctx.idx = idx
        out = ops.cast(zq, z.dtype).view(B, hz, wz, D)
        return out, loss3[0:1].clone()

    @staticmethod
    def backward(ctx, dzq, dloss):
        zf, zq, dE_unit = ctx.saved_tensors
        B, hz, wz, D = ctx.shape
        P = B * hz * wz
        dloss = dloss.to(torch.float32).contiguous()
        dz = torch.empty((B, hz, wz, D), dtype=ctx.dt, device=zf.device)
        dzq = None if dzq is None else dzq.contiguous()
        call("rdeic_vq_z_grad", zf.data_ptr(), zq.data_ptr(), None if dzq is None else dzq.data_ptr(), P * D,
             dloss.data_ptr(), float(ctx.beta * 2.0 / (P * D)), dz.data_ptr(), _dt(dz), _sp())
        dE = torch.empty_like(dE_unit)
        call("rdeic_scale_dev", dE_unit.data_ptr(), dE_unit.numel(), dloss.data_ptr(), dE.data_ptr(), 0, _sp())
        return dz, dE, None, None, None, None


def adamw_(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int, lr: float,
           betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2) -> None:
    """torch.optim.AdamW update of flat fp32 buffers in place (configure_optimizers, rdeic.py:763-772)."""
    for t in (p, g, m, v):
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("adamw_ expects contiguous fp32 buffers")
    call("rdeic_adamw", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), float(lr), float(betas[0]),
         float(betas[1]), float(eps), float(weight_decay), int(step), _sp())


def bpp_from_sum(S: torch.Tensor, num_pixels: int) -> torch.Tensor:
    """sum(log(lik)) / (-ln 2 * num_pixels)  (model/rdeic.py:684)."""
    return S / (-math.log(2) * num_pixels)
