"""The RDEIC compressor (model/compression.py, model/compression_modules.py, utils/ckbd.py)
on the HIP kernels + host C++ coders, batched over images.

Nets (NHWC, reference parameter names under `preprocess_model.`):
  g_a  Encoder        compression_modules.py:7-24   (ResidualBlock / WithStride, res_blk.py:6-93)
  hyper_enc / dec     compression_modules.py:47-73  (ResidualBlockUpsample = subpel 1x1 + PixelShuffle,
                                                     fused into the conv store)
  ChannelContextEX    compression_modules.py:76-89  (5x5 convs + exact GELU)
  EntropyParametersEX compression_modules.py:91-104 (1x1 convs + GELU), local_context 5x5
  VectorQuantiser.quant / get_codebook_entry        compression_modules.py:309-338
  g_s Decoder + out   compression_modules.py:27-44, compression.py:21
Entropy stage (10 slices x {anchor, non-anchor}, compression.py:171-203 / 233-264):
  params -> rdeic_ckbd_encode (squeeze, build_indexes, round, dequantise, unsqueeze in one
  kernel) -> per-image symbol/index lists in the reference order -> C++ rANS (one stream per
  image, host threads). Torch.cat of [local_ctx, channel_ctx, hyper_params] is never
  materialised: producers write into channel slices of one context buffer and the first
  entropy-parameter conv gathers its two input segments directly.
The reference codes batch 1 per call (utils/ckbd.py:140 hard-codes batch 1 on decode); every
kernel here is batch-invariant (fixed reduction order), so a batched call produces exactly the
per-image streams and reconstructions of B single-image calls.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import coders, ops
from .params import ParamStore

LEAK = 0.01


class Compression:
    def __init__(self, store: ParamStore, in_nc: int, out_nc: int, N: int, M: int, slice_num: int,
                 slice_ch: Sequence[int], codebook_size: int, prefix: str = "preprocess_model."):
        self.store, self.p = store, prefix
        self.N, self.M = N, M
        self.slice_num, self.slice_ch = slice_num, list(slice_ch)
        self.slice_off = [sum(self.slice_ch[:i]) for i in range(slice_num)]
        self.codebook_size = codebook_size
        p = prefix
        d = store
        # g_a
        self.g_a = []
        spec = [("rb", in_nc, M), ("rb", M, M), ("rb", M, M), ("rb", M, M), ("rbs", M, M), ("rb", M, M),
                ("rb", M, M), ("rb", M, M)]
        for i, (kind, ci, co) in enumerate(spec):
            self.g_a.append(self._declare_block(f"{p}encoder.g_a.{i}", kind, ci, co))
        d.declare_conv(f"{p}encoder.g_a.8", M, M, 3)
        self.g_a.append((f"{p}encoder.g_a.8", "conv", M, M))
        self.hyper_enc = [self._declare_block(f"{p}hyper_enc.hyper_enc.{i}", k, ci, co) for i, (k, ci, co) in
                          enumerate([("rb", M, N), ("rb", N, N), ("rbs", N, N), ("rbs", N, N)])]
        self.hyper_dec = [self._declare_block(f"{p}hyper_dec.hyper_dec.{i}", k, ci, co) for i, (k, ci, co) in
                          enumerate([("rbu", N, M), ("rbu", M, M), ("rb", M, M * 3 // 2), ("rb", M * 3 // 2, M * 2)])]
        d.declare_conv(f"{p}decoder.g_s.0", M, M, 3)
        self.g_s = [(f"{p}decoder.g_s.0", "conv", M, M)]
        for i, (k, ci, co) in enumerate([("rb", M, M)] * 3 + [("rbu", M, M)] + [("rb", M, M)] * 4):
            self.g_s.append(self._declare_block(f"{p}decoder.g_s.{i + 1}", k, ci, co))
        d.declare_conv(f"{p}out", out_nc, M, 3)
        for i, c in enumerate(self.slice_ch):
            d.declare_conv(f"{p}local_context.{i}", 2 * c, c, 5)
            if i:
                cin = sum(self.slice_ch[:i])
                d.declare_conv(f"{p}channel_context.{i}.fushion.0", 224, cin, 5)
                d.declare_conv(f"{p}channel_context.{i}.fushion.2", 128, 224, 5)
                d.declare_conv(f"{p}channel_context.{i}.fushion.4", 2 * c, 128, 5)
            for nm, cin in (("entropy_parameters_anchor", 2 * M + (2 * c if i else 0)),
                            ("entropy_parameters_nonanchor", 2 * M + (4 * c if i else 2 * c))):
                out = 2 * c
                d.declare_conv(f"{p}{nm}.{i}.fusion.0", out * 5 // 3, cin, 1)
                d.declare_conv(f"{p}{nm}.{i}.fusion.2", out * 4 // 3, out * 5 // 3, 1)
                d.declare_conv(f"{p}{nm}.{i}.fusion.4", out, out * 4 // 3, 1)
        d.declare(f"{p}quantize.embedding.weight", (codebook_size, N))
        self.tables = None
        self._en = None

    def _declare_block(self, pre, kind, ci, co):
        d = self.store
        if kind == "rb":
            d.declare_conv(pre + ".conv1", co, ci, 3)
            d.declare_conv(pre + ".conv2", co, co, 3)
            if ci != co:
                d.declare_conv(pre + ".adaptor", co, ci, 1)
        elif kind == "rbs":
            d.declare_conv(pre + ".conv1", co, ci, 3)
            d.declare_conv(pre + ".conv2", co, co, 3)
            d.declare_conv(pre + ".downsample", co, ci, 1)
        elif kind == "rbu":
            d.declare_conv(pre + ".subpel_conv.0", co * 4, ci, 1)
            d.declare_conv(pre + ".conv", co, co, 3)
            d.declare_conv(pre + ".upsample.0", co * 4, ci, 1)
        return (pre, kind, ci, co)

    # ------------------------------------------------------------------ tables
    def update(self, scale_table=None, force: bool = False):
        """GaussianConditional.update_scale_table(get_scale_table()) (compression.py:275-280)."""
        if self.tables is None or force or scale_table is not None:
            self.tables = coders.GaussianTables(scale_table)
        return True

    # ------------------------------------------------------------------ nets
    def _block(self, blk, x):
        pre, kind, ci, co = blk
        s = self.store
        if kind == "conv":
            return ops.conv2d(x, s.conv(pre))
        if kind == "rb":
            identity = x if ci == co else ops.conv2d(x, s.conv(pre + ".adaptor"))
            out = ops.conv2d(x, s.conv(pre + ".conv1"), act=ops.LEAKY, slope=LEAK)
            return ops.conv2d(out, s.conv(pre + ".conv2"), act=ops.LEAKY, slope=LEAK, res=identity)
        if kind == "rbs":
            out = ops.conv2d(x, s.conv(pre + ".conv1", stride=2, pad=1), act=ops.LEAKY, slope=LEAK)
            identity = ops.conv2d(x, s.conv(pre + ".downsample", stride=2, pad=0))
            return ops.conv2d(out, s.conv(pre + ".conv2"), act=ops.LEAKY, slope=0.1, res=identity)
        if kind == "rbu":
            out = ops.conv2d(x, s.conv(pre + ".subpel_conv.0"), pixel_shuffle=True, act=ops.LEAKY, slope=LEAK)
            identity = ops.conv2d(x, s.conv(pre + ".upsample.0"), pixel_shuffle=True)
            return ops.conv2d(out, s.conv(pre + ".conv"), act=ops.LEAKY, slope=0.1, res=identity)
        raise ValueError(kind)

    def _seq(self, blocks, x):
        for b in blocks:
            x = self._block(b, x)
        return x

    def _ep(self, name: str, i: int, x: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
        s, p = self.store, self.p
        h = ops.conv2d(x, s.conv(f"{p}{name}.{i}.fusion.0"), x2=x2, act=ops.GELU)
        h = ops.conv2d(h, s.conv(f"{p}{name}.{i}.fusion.2"), act=ops.GELU)
        return ops.conv2d(h, s.conv(f"{p}{name}.{i}.fusion.4"))

    def _channel_ctx(self, i: int, yhat_prefix: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
        s, p = self.store, self.p
        h = ops.conv2d(yhat_prefix, s.conv(f"{p}channel_context.{i}.fushion.0"), act=ops.GELU)
        h = ops.conv2d(h, s.conv(f"{p}channel_context.{i}.fushion.2"), act=ops.GELU)
        return ops.conv2d(h, s.conv(f"{p}channel_context.{i}.fushion.4"), out=out)

    # ------------------------------------------------------------------ VQ
    def _codebook(self) -> torch.Tensor:
        return self.store.get(self.p + "quantize.embedding.weight")

    def vq_quant(self, z: torch.Tensor):
        """VectorQuantiser.quant: first-argmin over (|z|^2 + |e|^2) - 2 z.e in fp32."""
        B, hz, wz, N = z.shape
        rows = B * hz * wz
        E = self._codebook()
        zf = ops.cast(z.contiguous(), torch.float32).view(rows, N)
        zn = torch.empty(rows, dtype=torch.float32, device=z.device)
        ops.call("rdeic_row_sqnorm", zf.data_ptr(), rows, N, N, zn.data_ptr(), 0, ops.stream_ptr())
        if self._en is None or self._en.device != z.device:
            self._en = torch.empty(E.shape[0], dtype=torch.float32, device=z.device)
            ops.call("rdeic_row_sqnorm", E.data_ptr(), E.shape[0], N, N, self._en.data_ptr(), 0, ops.stream_ptr())
        dot = ops.linear(zf, self.store.conv(self.p + "quantize.embedding", dtype=torch.float32))
        idx = torch.empty(rows, dtype=torch.int32, device=z.device)
        ops.call("rdeic_vq_argmin", dot.data_ptr(), zn.data_ptr(), self._en.data_ptr(), rows, E.shape[0],
                 idx.data_ptr(), ops.stream_ptr())
        return self.codebook_entry(idx, B, hz, wz), idx.view(B, hz, wz)

    def codebook_entry(self, idx: torch.Tensor, B: int, hz: int, wz: int) -> torch.Tensor:
        E = self._codebook()
        N = E.shape[1]
        zq = torch.empty((B, hz, wz, N), dtype=self.store.compute_dtype, device=E.device)
        ops.call("rdeic_gather_rows", E.data_ptr(), N, idx.contiguous().data_ptr(), B * hz * wz, N, zq.data_ptr(), N,
                 ops.dt_code(zq), ops.stream_ptr())
        return zq

    # ------------------------------------------------------------------ entropy stages
    def _pinned(self, key: str, n: int, dtype=torch.int32) -> torch.Tensor:
        """Reusable page-locked host staging buffer (>= n elements) for the coder round trips."""
        cache = self.__dict__.setdefault("_pin_cache", {})
        buf = cache.get(key)
        if buf is None or buf.numel() < n or buf.dtype != dtype:
            buf = torch.empty(max(n, 1), dtype=dtype, pin_memory=True)
            cache[key] = buf
        return buf[:n]

    def stage_sizes(self, hy: int, wy: int) -> List[int]:
        sizes = []
        for c in self.slice_ch:
            sizes += [c * hy * (wy // 2)] * 2
        return sizes

    def _stage_common(self, hy, wy, B, device, dt):
        yhat = torch.empty((B, hy, wy, self.M), dtype=dt, device=device)
        cmax = max(self.slice_ch)
        ctx = torch.empty((B, hy, wy, 4 * cmax), dtype=dt, device=device)
        anchor = torch.empty((B, hy, wy, cmax), dtype=dt, device=device)
        return yhat, ctx, anchor

    def _run_stages(self, hyper, B, hy, wy, emit):
        """Drive the 20 checkerboard stages. emit(i, phase, params, c, off, yhat_slice, anchor_buf)
        produces the dequantised slice values (encode: from y; decode: from the bitstream)."""
        dt, dev = hyper.dtype, hyper.device
        yhat, ctxbuf, anchor_full = self._stage_common(hy, wy, B, dev, dt)
        off = 0
        for i, c in enumerate(self.slice_ch):
            s0 = self.slice_off[i]
            ctx = ctxbuf[..., :4 * c]
            anchor = anchor_full[..., :c]
            if i == 0:
                pa = self._ep("entropy_parameters_anchor", 0, hyper, None)
            else:
                self._channel_ctx(i, yhat[..., :s0], out=ctx[..., 2 * c:4 * c])
                pa = self._ep("entropy_parameters_anchor", i, ctx[..., 2 * c:4 * c], hyper)
            emit(i, 0, pa, c, off, yhat[..., s0:s0 + c], anchor)
            off += c * hy * (wy // 2)
            ops.conv2d(anchor, self.store.conv(f"{self.p}local_context.{i}"), out=ctx[..., :2 * c])
            pn = self._ep("entropy_parameters_nonanchor", i, ctx[..., :(4 * c if i else 2 * c)], hyper)
            emit(i, 1, pn, c, off, yhat[..., s0:s0 + c], None)
            off += c * hy * (wy // 2)
        return yhat

    # ------------------------------------------------------------------ compress / decompress
    @torch.no_grad()
    def compress(self, h: torch.Tensor) -> List[dict]:
        """h: NHWC [B, H/8, W/8, 512] (compute dtype). Returns one reference-format dict per image:
        {"strings": [[y_string], [z_string]], "shape": (zh, zw)} (compression.py:151-213)."""
        self.update()
        s = self.store
        B = h.shape[0]
        y = self._seq(self.g_a, h)
        z = self._seq(self.hyper_enc, y)
        z_q, z_idx = self.vq_quant(z)
        hyper = self._seq(self.hyper_dec, z_q)
        _, hy, wy, _ = y.shape
        total = sum(self.stage_sizes(hy, wy))
        sym = torch.empty((B, total), dtype=torch.int32, device=h.device)
        idx = torch.empty((B, total), dtype=torch.int32, device=h.device)
        table = self.tables.device_scale_table(h.device)
        dtc = ops.dt_code(h)

        def emit(i, phase, params, c, off, yhat_slice, anchor):
            s0 = self.slice_off[i]
            ys = y[..., s0:s0 + c]
            ops.call("rdeic_ckbd_encode", ys.data_ptr(), ops.pix_ld(ys), params.data_ptr(), ops.pix_ld(params), B, hy,
                     wy, c, phase, table.data_ptr(), table.numel(), float(coders.SCALE_BOUND), sym.data_ptr(),
                     idx.data_ptr(), total, off, yhat_slice.data_ptr(), ops.pix_ld(yhat_slice),
                     None if anchor is None else anchor.data_ptr(), 0 if anchor is None else ops.pix_ld(anchor), dtc,
                     ops.stream_ptr())

        self._run_stages(hyper, B, hy, wy, emit)
        sym_p = self._pinned("enc_sym", B * total).view(B, total)
        idx_p = self._pinned("enc_idx", B * total).view(B, total)
        sym_p.copy_(sym, non_blocking=True)
        idx_p.copy_(idx, non_blocking=True)
        zi = z_idx.cpu().numpy()  # synchronises the stream: the pinned copies above are complete
        sym_h, idx_h = sym_p.numpy(), idx_p.numpy()
        y_strings = coders.rans_encode_batch(sym_h, idx_h, self.tables)
        hz, wz = z.shape[1], z.shape[2]
        out = []
        for b in range(B):
            z_str = coders.ac_encode_uniform(zi[b], self.codebook_size)
            out.append({"strings": [[y_strings[b]], [z_str]], "shape": (hz, wz)})
        return out

    @torch.no_grad()
    def decompress(self, strings_list: Sequence[Sequence[Sequence[bytes]]], shape: Tuple[int, int],
                   device="cuda") -> Tuple[torch.Tensor, torch.Tensor]:
        """strings_list[b] = [[y_string], [z_string]] for image b (all of one latent shape).
        Returns (c_latent fp32 NHWC [B,h,w,4], guide_hint NHWC [B,h,w,M]) (compression.py:215-273)."""
        self.update()
        B = len(strings_list)
        hz, wz = int(shape[0]), int(shape[1])
        zi = np.stack([coders.ac_decode_uniform(st[1][0], hz * wz, self.codebook_size) for st in strings_list])
        z_idx = torch.from_numpy(zi.astype(np.int32)).to(device)
        z_q = self.codebook_entry(z_idx, B, hz, wz)
        hyper = self._seq(self.hyper_dec, z_q)
        _, hy, wy, _ = hyper.shape
        decs = [coders.RansDecoder(st[0][0]) for st in strings_list]
        nmax = B * max(self.stage_sizes(hy, wy))
        self._pinned("dec_idx", nmax), self._pinned("dec_sym", nmax)  # size once: no regrowth mid-loop
        table = self.tables.device_scale_table(hyper.device)
        dtc = ops.dt_code(hyper)

        def emit(i, phase, params, c, off, yhat_slice, anchor):
            n = c * hy * (wy // 2)
            idx = torch.empty((B, n), dtype=torch.int32, device=hyper.device)
            ops.call("rdeic_ckbd_indexes", params.data_ptr(), ops.pix_ld(params), B, hy, wy, c, phase,
                     table.data_ptr(), table.numel(), float(coders.SCALE_BOUND), idx.data_ptr(), n, 0, dtc,
                     ops.stream_ptr())
            idx_p = self._pinned("dec_idx", B * n).view(B, n)
            idx_p.copy_(idx, non_blocking=True)
            torch.cuda.current_stream(hyper.device).synchronize()
            sym_p = self._pinned("dec_sym", B * n).view(B, n)
            coders.rans_decode_batch(decs, idx_p.numpy(), self.tables, out=sym_p.numpy())
            sym = sym_p.to(hyper.device, non_blocking=True)
            ops.call("rdeic_ckbd_dequant", sym.data_ptr(), params.data_ptr(), ops.pix_ld(params), B, hy, wy, c, phase,
                     n, 0, yhat_slice.data_ptr(), ops.pix_ld(yhat_slice),
                     None if anchor is None else anchor.data_ptr(), 0 if anchor is None else ops.pix_ld(anchor), dtc,
                     ops.stream_ptr())

        yhat = self._run_stages(hyper, B, hy, wy, emit)
        for d in decs:
            d.close()
        guide_hint = self._seq(self.g_s, yhat)
        c_latent = ops.conv2d(guide_hint, self.store.conv(self.p + "out"), out_f32=True)
        return c_latent, guide_hint
