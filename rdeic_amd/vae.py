"""AutoencoderKL encoder (forward_hc) and decoder on the HIP kernels, NHWC.

Mirrors ldm/modules/diffusionmodules/model.py (ResnetBlock :92-151, AttnBlock :154-205,
Downsample :70-89 with its asymmetric (0,1,0,1) pad, Upsample :52-67, Encoder.forward_hc
:551-577, Decoder.forward :653-686) and ldm/models/autoencoder.py (encode_hc :91-95,
decode :97-100) with the reference's parameter names under `first_stage_model.`.

encode_hc's conv_out / quant_conv / DiagonalGaussianDistribution results are discarded by the
only caller on the hot path (RDEIC.apply_condition_compress, model/rdeic.py:661), so only
`c = swish(norm_out(h))` is produced (the parameters are still declared for checkpoint
compatibility). The latent scale (x 0.18215, rdeic.py:662) is fused into that last kernel.
"""
from __future__ import annotations

import torch

from . import ops
from .params import ParamStore

GN_EPS = 1e-6


class AutoencoderKL:
    def __init__(self, store: ParamStore, dd: dict, embed_dim: int, prefix: str = "first_stage_model."):
        self.store, self.prefix, self.dd = store, prefix, dd
        ch, chm, nrb = dd["ch"], dd["ch_mult"], dd["num_res_blocks"]
        zc = dd["z_channels"]
        self.nres = len(chm)
        e = prefix + "encoder."
        store.declare_conv(e + "conv_in", ch, dd["in_channels"], 3)
        in_chm = (1,) + tuple(chm)
        self.enc_blocks = []
        block_in = ch
        for i in range(self.nres):
            block_in = ch * in_chm[i]
            block_out = ch * chm[i]
            lvl = []
            for j in range(nrb):
                lvl.append(self._declare_resnet(f"{e}down.{i}.block.{j}", block_in, block_out))
                block_in = block_out
            down = None
            if i != self.nres - 1:
                down = f"{e}down.{i}.downsample.conv"
                store.declare_conv(down, block_in, block_in, 3)
            self.enc_blocks.append((lvl, down))
        self.enc_mid = (self._declare_resnet(e + "mid.block_1", block_in, block_in),
                        self._declare_attn(e + "mid.attn_1", block_in),
                        self._declare_resnet(e + "mid.block_2", block_in, block_in))
        store.declare_norm(e + "norm_out", block_in)
        store.declare_conv(e + "conv_out", 2 * zc if dd["double_z"] else zc, block_in, 3)
        self.enc_out_ch = block_in
        store.declare_conv(prefix + "quant_conv", 2 * embed_dim, 2 * zc, 1)
        store.declare_conv(prefix + "post_quant_conv", zc, embed_dim, 1)
        d = prefix + "decoder."
        block_in = ch * chm[-1]
        store.declare_conv(d + "conv_in", block_in, zc, 3)
        self.dec_mid = (self._declare_resnet(d + "mid.block_1", block_in, block_in),
                        self._declare_attn(d + "mid.attn_1", block_in),
                        self._declare_resnet(d + "mid.block_2", block_in, block_in))
        self.dec_blocks = []
        for i in reversed(range(self.nres)):
            block_out = ch * chm[i]
            lvl = []
            for j in range(nrb + 1):
                lvl.append(self._declare_resnet(f"{d}up.{i}.block.{j}", block_in, block_out))
                block_in = block_out
            up = None
            if i != 0:
                up = f"{d}up.{i}.upsample.conv"
                store.declare_conv(up, block_in, block_in, 3)
            self.dec_blocks.append((lvl, up))
        store.declare_norm(d + "norm_out", block_in)
        store.declare_conv(d + "conv_out", dd["out_ch"], block_in, 3)

    # ------------------------------------------------------------------ declarations
    def _declare_resnet(self, pre, cin, cout):
        s = self.store
        s.declare_norm(pre + ".norm1", cin)
        s.declare_conv(pre + ".conv1", cout, cin, 3)
        s.declare_norm(pre + ".norm2", cout)
        s.declare_conv(pre + ".conv2", cout, cout, 3)
        if cin != cout:
            s.declare_conv(pre + ".nin_shortcut", cout, cin, 1)
        return (pre, cin, cout)

    def _declare_attn(self, pre, c):
        s = self.store
        s.declare_norm(pre + ".norm", c)
        for n in ("q", "k", "v", "proj_out"):
            s.declare_conv(f"{pre}.{n}", c, c, 1)
        return (pre, c)

    # ------------------------------------------------------------------ blocks
    def resnet(self, blk, x):
        pre, cin, cout = blk
        s = self.store
        ab1 = ops.group_norm_ab(x, s.get(pre + ".norm1.weight"), s.get(pre + ".norm1.bias"), 32, GN_EPS)
        h = ops.conv2d(x, s.conv(pre + ".conv1"), gn=ab1, gn_silu=True, stats=True)
        ab2 = ops.group_norm_ab(h, s.get(pre + ".norm2.weight"), s.get(pre + ".norm2.bias"), 32, GN_EPS)
        skip = x if cin == cout else ops.conv2d(x, s.conv(pre + ".nin_shortcut"))
        # every ResnetBlock output feeds a GroupNorm (next block, AttnBlock or norm_out)
        return ops.conv2d(h, s.conv(pre + ".conv2"), gn=ab2, gn_silu=True, res=skip, stats=True)

    def attn(self, blk, x):
        pre, c = blk
        s = self.store
        B, H, W_, C = x.shape
        L = H * W_
        ab = ops.group_norm_ab(x, s.get(pre + ".norm.weight"), s.get(pre + ".norm.bias"), 32, GN_EPS)
        qkv = ops.conv2d(x, s.conv_cat([pre + ".q", pre + ".k", pre + ".v"]), gn=ab, gn_silu=False)
        qkv = qkv.view(B * L, 3 * C)
        o = torch.empty((B * L, C), dtype=x.dtype, device=x.device)
        if x.dtype == torch.bfloat16 and C == 512 and L % 32 == 0 and ops.VAE_FLASH_ATTENTION:
            # flash kernel (attention.hip attn512_kernel): no score matrix in HBM
            ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, batch=B, heads=1, lq=L, lk=L, dh=C,
                          scale=int(C) ** (-0.5))
        else:  # fp32 parity mode: the materialised GEMM -> softmax -> GEMM (reference op order)
            ops.attention_single_head_materialized(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, batch=B,
                                                   length=L, dim=C, scale=int(C) ** (-0.5))
        out = ops.linear(o, s.conv(pre + ".proj_out"), res=x.contiguous().view(B * L, C), stats_hw=L,
                          images=B)
        return ops.tokens_to_nhwc(out, B, H, W_)

    # ------------------------------------------------------------------ passes
    def encode_hc(self, x: torch.Tensor, out_mul: float = 1.0) -> torch.Tensor:
        """x: NHWC compute-dtype image in [-1, 1] ([B,H,W,3]); returns c * out_mul, [B,H/8,W/8,512]."""
        return self._encode(x, out_mul, moments=False)

    def encode_hc_moments(self, x: torch.Tensor, out_mul: float = 1.0):
        """encode_hc + the posterior moments (autoencoder.py:91-95): (c * out_mul, moments fp32 NHWC
        [B,H/8,W/8,8] = quant_conv(conv_out(c))) for the fine-tune step's x_start sample."""
        return self._encode(x, out_mul, moments=True)

    def _encode(self, x: torch.Tensor, out_mul: float, moments: bool):
        s = self.store
        e = self.prefix + "encoder."
        h = ops.conv2d(x, s.conv(e + "conv_in", cin_pad=x.shape[3] if x.shape[3] > 3 else None), stats=True)
        for lvl, down in self.enc_blocks:
            for blk in lvl:
                h = self.resnet(blk, h)
            if down is not None:
                Hh, Ww = h.shape[1], h.shape[2]
                h = ops.conv2d(h, s.conv(down, stride=2, pad=0), pad_t=0, pad_l=0, out_hw=(Hh // 2, Ww // 2),
                               stats=True)
        h = self.resnet(self.enc_mid[0], h)
        h = self.attn(self.enc_mid[1], h)
        h = self.resnet(self.enc_mid[2], h)
        ab = ops.group_norm_ab(h, s.get(e + "norm_out.weight"), s.get(e + "norm_out.bias"), 32, GN_EPS)
        if not moments:
            return ops.group_norm_apply(h, ab, silu=True, out_mul=out_mul)
        c = ops.group_norm_apply(h, ab, silu=True)
        hc = ops.conv2d(c, s.conv(e + "conv_out"), out_f32=True)
        mom = ops.conv2d(hc, s.conv(self.prefix + "quant_conv", dtype=torch.float32))
        if out_mul != 1.0:
            c = ops.group_norm_apply(h, ab, silu=True, out_mul=out_mul)
        return c, mom

    def decode(self, z: torch.Tensor, out_f32: bool = True) -> torch.Tensor:
        """z: compute-dtype NHWC [B,h,w,4] (already divided by the scale factor); returns NHWC [B,8h,8w,3]."""
        s = self.store
        d = self.prefix + "decoder."
        z = ops.conv2d(z, s.conv(self.prefix + "post_quant_conv"))
        h = ops.conv2d(z, s.conv(d + "conv_in"), stats=True)
        h = self.resnet(self.dec_mid[0], h)
        h = self.attn(self.dec_mid[1], h)
        h = self.resnet(self.dec_mid[2], h)
        for lvl, up in self.dec_blocks:
            for blk in lvl:
                h = self.resnet(blk, h)
            if up is not None:
                h = ops.conv2d(h, s.conv(up), up2=True, stats=True)
        ab = ops.group_norm_ab(h, s.get(d + "norm_out.weight"), s.get(d + "norm_out.bias"), 32, GN_EPS)
        return ops.conv2d(h, s.conv(d + "conv_out"), gn=ab, gn_silu=True, out_f32=out_f32)
