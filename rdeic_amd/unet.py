"""SD-2.1 UNet + RDEIC control branch (NoiseEstimator) on the HIP kernels, NHWC.

Mirrors, block for block and with the reference's parameter names:
  UNetModel            ldm/modules/diffusionmodules/openaimodel.py:421-807
  ResBlock             openaimodel.py:162-274 (control copy: model/rdeic.py:487-598)
  SpatialTransformer   ldm/modules/attention.py:288-350 (BasicTransformerBlock :255-285,
                       CrossAttention :153-203, GEGLU :49-56)
  ControlModule        model/rdeic.py:237-462 (0.2x width copy of the encoder half)
  NoiseEstimator       model/rdeic.py:38-212 (zero convs, forward :174-212)

Kernel mapping per ResBlock: GN stats -> conv3x3 with fused GN-affine+SiLU prologue and
timestep-embedding epilogue -> GN stats -> conv3x3 with fused GN+SiLU prologue and the skip
(identity or 1x1 conv) as residual epilogue. Torch.cat of the decoder skip is never
materialised: the conv gathers from both tensors and GN statistics run per segment.
All 25 ResBlocks' emb_layers are one fp32 GEMM (stacked weights) per network.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import ops
from .params import ParamStore


def find_denominator(number: int, start: int) -> int:
    """Largest divisor of `number` that is <= start (model/rdeic.py:464-471)."""
    if start >= number:
        return number
    while start != 0:
        if number % start == 0:
            return start
        start -= 1
    return 1


@dataclass
class ResBlock:
    prefix: str
    cin: int
    cout: int
    gn_in: int
    gn_out: int
    emb_off: int = 0


@dataclass
class SpatialTransformer:
    prefix: str
    ch: int
    heads: int
    dh: int
    gn: int


@dataclass
class Conv:
    prefix: str
    cin: int
    cout: int


@dataclass
class Down:
    prefix: str
    ch: int


@dataclass
class Up:
    prefix: str
    ch: int


class UNet:
    """The base UNetModel (control=False) or the ControlModule (control=True)."""

    def __init__(self, store: ParamStore, prefix: str, cfg: dict, control: bool = False):
        self.store, self.prefix, self.control = store, prefix, control
        mc0 = cfg["model_channels"]
        self.mc0 = mc0
        ted = mc0 * 4
        self.ted = ted
        ctx_dim = cfg["context_dim"]
        self.ctx_dim = ctx_dim
        store.declare_linear(prefix + "time_embed.0", ted, mc0)
        store.declare_linear(prefix + "time_embed.2", ted, ted)
        mc = int(mc0 * cfg["control_model_ratio"]) if control else mc0
        in_ch = cfg["in_channels"] + (cfg["hint_channels"] if control else 0)
        nhc = cfg["num_head_channels"]
        attn_res = cfg["attention_resolutions"]
        nrb = cfg["num_res_blocks"]
        mults = cfg["channel_mult"]
        self.resblocks: List[ResBlock] = []
        gn = (lambda c: find_denominator(c, 32)) if control else (lambda c: 32)

        def res(pre, cin, cout):
            rb = ResBlock(pre, cin, cout, gn(cin), gn(cout))
            store.declare_norm(pre + ".in_layers.0", cin)
            store.declare_conv(pre + ".in_layers.2", cout, cin, 3)
            store.declare_linear(pre + ".emb_layers.1", cout, ted)
            store.declare_norm(pre + ".out_layers.0", cout)
            store.declare_conv(pre + ".out_layers.3", cout, cout, 3)
            if cin != cout:
                store.declare_conv(pre + ".skip_connection", cout, cin, 1)
            self.resblocks.append(rb)
            return rb

        def st(pre, ch):
            nonlocal nhc_cur
            if control:
                nhc_cur = find_denominator(ch, nhc)
            heads, dh = ch // nhc_cur, nhc_cur
            inner = heads * dh
            store.declare_norm(pre + ".norm", ch)
            store.declare_linear(pre + ".proj_in", inner, ch)
            tb = pre + ".transformer_blocks.0"
            for a in ("attn1", "attn2"):
                kv_in = ch if a == "attn1" else ctx_dim
                store.declare_linear(f"{tb}.{a}.to_q", inner, ch, bias=False)
                store.declare_linear(f"{tb}.{a}.to_k", inner, kv_in, bias=False)
                store.declare_linear(f"{tb}.{a}.to_v", inner, kv_in, bias=False)
                store.declare_linear(f"{tb}.{a}.to_out.0", ch, inner)
            store.declare_linear(tb + ".ff.net.0.proj", inner * 8, inner)
            store.declare_linear(tb + ".ff.net.2", inner, inner * 4)
            for nn_ in ("norm1", "norm2", "norm3"):
                store.declare_norm(f"{tb}.{nn_}", inner)
            store.declare_linear(pre + ".proj_out", inner, ch)
            return SpatialTransformer(pre, ch, heads, dh, find_denominator(ch, 32))

        nhc_cur = nhc
        self.input_blocks: List[list] = []
        p0 = prefix + "input_blocks.0.0"
        store.declare_conv(p0, mc, in_ch, 3)
        self.input_blocks.append([Conv(p0, in_ch, mc)])
        chans, ch, ds, idx = [mc], mc, 1, 1
        for level, mult in enumerate(mults):
            for _ in range(nrb):
                layers = [res(f"{prefix}input_blocks.{idx}.0", ch, mult * mc)]
                ch = mult * mc
                if ds in attn_res:
                    layers.append(st(f"{prefix}input_blocks.{idx}.1", ch))
                self.input_blocks.append(layers)
                chans.append(ch)
                idx += 1
            if level != len(mults) - 1:
                pre = f"{prefix}input_blocks.{idx}.0.op"
                store.declare_conv(pre, ch, ch, 3)
                self.input_blocks.append([Down(pre, ch)])
                chans.append(ch)
                ds *= 2
                idx += 1
        self.enc_out_ch = list(chans)
        self.middle = [res(prefix + "middle_block.0", ch, ch), st(prefix + "middle_block.1", ch),
                       res(prefix + "middle_block.2", ch, ch)]
        self.mid_ch = ch
        self.output_blocks: List[list] = []
        self.dec_out_ch: List[int] = []
        if not control:
            k = 0
            for level, mult in list(enumerate(mults))[::-1]:
                for i in range(nrb + 1):
                    ich = chans.pop()
                    layers = [res(f"{prefix}output_blocks.{k}.0", ch + ich, mc * mult)]
                    ch = mc * mult
                    if ds in attn_res:
                        layers.append(st(f"{prefix}output_blocks.{k}.1", ch))
                    if level and i == nrb:
                        pre = f"{prefix}output_blocks.{k}.{len(layers)}.conv"
                        store.declare_conv(pre, ch, ch, 3)
                        layers.append(Up(pre, ch))
                        ds //= 2
                    self.output_blocks.append(layers)
                    self.dec_out_ch.append(ch)
                    k += 1
            store.declare_norm(prefix + "out.0", ch)
            store.declare_conv(prefix + "out.2", cfg["out_channels"], mc, 3)
        off = 0
        for rb in self.resblocks:
            rb.emb_off = off
            off += rb.cout
        self.emb_total = off

    # ------------------------------------------------------------------ forward pieces
    def time_embed(self, temb: torch.Tensor) -> torch.Tensor:
        """SiLU(time_embed(t_emb)) @ stacked emb_layers -> [B, sum(cout)] fp32 (one GEMM)."""
        s = self.store
        B = temb.shape[0]  # one row per image
        e = ops.linear(temb, s.conv(self.prefix + "time_embed.0", dtype=torch.float32), act=ops.SILU, images=B)
        e = ops.linear(e, s.conv(self.prefix + "time_embed.2", dtype=torch.float32), act=ops.SILU, images=B)
        stacked = s.conv_cat([rb.prefix + ".emb_layers.1" for rb in self.resblocks], dtype=torch.float32)
        return ops.linear(e, stacked, images=B)

    def resblock(self, rb: ResBlock, x: torch.Tensor, emb_all: torch.Tensor,
                 x2: Optional[torch.Tensor] = None, stats: bool = False) -> torch.Tensor:
        """stats: the output feeds a GroupNorm (its statistics come fused with the last conv)."""
        s = self.store
        ab1 = ops.group_norm_ab(x, s.get(rb.prefix + ".in_layers.0.weight"), s.get(rb.prefix + ".in_layers.0.bias"),
                                rb.gn_in, 1e-5, x2=x2, defer=True)
        h = ops.conv2d(x, s.conv(rb.prefix + ".in_layers.2"), x2=x2, gn=ab1, gn_silu=True,
                       emb=emb_all[:, rb.emb_off:rb.emb_off + rb.cout], stats=True)
        ab2 = ops.group_norm_ab(h, s.get(rb.prefix + ".out_layers.0.weight"),
                                s.get(rb.prefix + ".out_layers.0.bias"), rb.gn_out, 1e-5, defer=True)
        if rb.cin != rb.cout:
            skip = ops.conv2d(x, s.conv(rb.prefix + ".skip_connection"), x2=x2)
        else:
            if x2 is not None:
                raise ValueError("identity skip with a concatenated input")
            skip = x
        return ops.conv2d(h, s.conv(rb.prefix + ".out_layers.3"), gn=ab2, gn_silu=True, res=skip, stats=stats)

    def transformer(self, t: SpatialTransformer, x: torch.Tensor, ctx_kv_in: torch.Tensor, ctx_batch: int,
                    ctx_len: int, stats: bool = False) -> torch.Tensor:
        s = self.store
        B, H, W_, C = x.shape
        L = H * W_
        rows = B * L
        tb = t.prefix + ".transformer_blocks.0"
        ab = ops.group_norm_ab(x, s.get(t.prefix + ".norm.weight"), s.get(t.prefix + ".norm.bias"), t.gn, 1e-6,
                               defer=True)
        h4 = ops.conv2d(x, s.conv(t.prefix + ".proj_in"), gn=ab, gn_silu=False)
        h = h4.view(rows, C)
        scale = t.dh ** -0.5
        # LayerNorms folded into the linears they feed (bf16): row statistics only, no normalised tensor
        fold = x.dtype == torch.bfloat16 and ops.LN_FOLD and C % 64 == 0
        # self-attention
        qkv_names = [tb + ".attn1.to_q", tb + ".attn1.to_k", tb + ".attn1.to_v"]
        if fold:
            qkv = ops.linear(h, s.conv_ln(qkv_names, tb + ".norm1"), ln_rows=ops.layer_norm_rowstats(h), images=B)
        else:
            n1 = ops.layer_norm(h, s.get(tb + ".norm1.weight"), s.get(tb + ".norm1.bias"))
            qkv = ops.linear(n1, s.conv_cat(qkv_names), images=B)
        o = torch.empty((rows, C), dtype=x.dtype, device=x.device)
        ops.attention(qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:], o, batch=B, heads=t.heads, lq=L, lk=L, dh=t.dh,
                      scale=scale)
        h = ops.linear(o, s.conv(tb + ".attn1.to_out.0"), res=h, images=B)
        # cross-attention against the text context
        if fold:
            q = ops.linear(h, s.conv_ln([tb + ".attn2.to_q"], tb + ".norm2"), ln_rows=ops.layer_norm_rowstats(h),
                           images=B)
        else:
            n2 = ops.layer_norm(h, s.get(tb + ".norm2.weight"), s.get(tb + ".norm2.bias"))
            q = ops.linear(n2, s.conv(tb + ".attn2.to_q"), images=B)
        kv = ops.linear(ctx_kv_in, s.conv_cat([tb + ".attn2.to_k", tb + ".attn2.to_v"]), images=ctx_batch)
        ops.attention(q, kv[:, :C], kv[:, C:], o, batch=B, heads=t.heads, lq=L, lk=ctx_len, dh=t.dh, scale=scale,
                      kv_bcast=(ctx_batch == 1 and B > 1))
        h = ops.linear(o, s.conv(tb + ".attn2.to_out.0"), res=h, images=B)
        # GEGLU feed-forward
        if fold and ops.GEGLU_FUSED:
            gg = ops.linear(h, s.conv_ln([tb + ".ff.net.0.proj"], tb + ".norm3", geglu=True),
                            ln_rows=ops.layer_norm_rowstats(h), geglu=True, images=B)
        else:
            n3 = ops.layer_norm(h, s.get(tb + ".norm3.weight"), s.get(tb + ".norm3.bias"))
            if x.dtype == torch.bfloat16 and ops.GEGLU_FUSED and C % 64 == 0:
                gg = ops.linear(n3, s.conv_geglu(tb + ".ff.net.0.proj"), geglu=True, images=B)  # one pass, half the writes
            else:
                gg = ops.geglu(ops.linear(n3, s.conv(tb + ".ff.net.0.proj"), images=B))
        h = ops.linear(gg, s.conv(tb + ".ff.net.2"), res=h, images=B)
        # proj_out + residual to the block input
        if not x.is_contiguous():
            raise ValueError("transformer input must be contiguous NHWC")
        out = ops.linear(h, s.conv(t.prefix + ".proj_out"), res=x.view(rows, C), stats_hw=L if stats else None,
                         images=B)
        return ops.tokens_to_nhwc(out, B, H, W_)

    def run_layers(self, layers, x, emb_all, ctx_rows, ctx_batch, ctx_len, x2=None, stats_last: bool = True):
        """Every layer's output but the last feeds the next layer's GroupNorm, so it carries fused
        statistics; the last one does when stats_last (its consumer is a GroupNorm too)."""
        s = self.store
        for li, layer in enumerate(layers):
            st = stats_last or li + 1 < len(layers)
            if isinstance(layer, Conv):
                x = ops.conv2d(x, s.conv(layer.prefix), x2=x2, stats=st)
                x2 = None
            elif isinstance(layer, ResBlock):
                x = self.resblock(layer, x, emb_all, x2=x2, stats=st)
                x2 = None
            elif isinstance(layer, SpatialTransformer):
                x = self.transformer(layer, x, ctx_rows, ctx_batch, ctx_len, stats=st)
            elif isinstance(layer, Down):
                x = ops.conv2d(x, s.conv(layer.prefix, stride=2, pad=1), stats=st)
            elif isinstance(layer, Up):
                x = ops.conv2d(x, s.conv(layer.prefix), up2=True, stats=st)
            else:
                raise TypeError(layer)
        return x


class NoiseEstimator:
    """model/rdeic.py:38-212 — base SD UNet + ControlModule + zero convs."""

    def __init__(self, store: ParamStore, unet_cfg: dict, control_cfg: dict,
                 base_prefix: str = "model.diffusion_model.", ctrl_prefix: str = "control_model."):
        self.store = store
        self.base = UNet(store, base_prefix, unet_cfg, control=False)
        self.ctrl = UNet(store, ctrl_prefix + "control_model.", control_cfg, control=True)
        self.model_channels = unet_cfg["model_channels"]
        self.control_scale = float(control_cfg.get("control_scale", 1.0))
        cp = ctrl_prefix
        enc_c, enc_b = self.ctrl.enc_out_ch, self.base.enc_out_ch
        self.enc_zero = [f"{cp}enc_zero_convs_out.{i}.0" for i in range(len(enc_c))]
        for i, pre in enumerate(self.enc_zero):
            store.declare_conv(pre, enc_b[i], enc_c[i], 1)
        self.mid_zero = f"{cp}middle_block_out.0"
        store.declare_conv(self.mid_zero, self.base.mid_ch, self.ctrl.mid_ch, 1)
        self.dec_zero = []
        for i in range(len(enc_c)):
            pre = f"{cp}dec_zero_convs_out.{i}.0"
            cout = self.base.mid_ch if i == 0 else self.base.dec_out_ch[i - 1]
            store.declare_conv(pre, cout, enc_c[-(i + 1)], 1)
            self.dec_zero.append(pre)
        # freqs of timestep_embedding (util.py:161-181), fp32 as torch computes them
        half = self.model_channels // 2
        import math
        self._freqs_cpu = torch.exp(-math.log(10000) * torch.arange(start=0, end=half, dtype=torch.float32) / half)
        self._freqs = None

    def _pad64(self, x: torch.Tensor) -> torch.Tensor:
        """x [B,h,w,c<64] -> [B,h,w,64] with channels c.. zero (the pad buffer is zeroed once per shape;
        only channels [0, c) are written per call, also under launch-plan replay)."""
        B, H, W_, c = x.shape
        key = (B, H, W_, x.dtype, ops.stream_ptr())
        cache = self.__dict__.setdefault("_pad_cache", {})
        buf = cache.get(key)
        if buf is None:
            buf = torch.zeros((B, H, W_, 64), dtype=x.dtype, device=x.device)
            cache[key] = buf
        xc = x.contiguous()
        ops.call("rdeic_act_fwd", xc.data_ptr(), B * H * W_, c, c, None, 0, 0, 0.0, buf.data_ptr(), 64,
                 ops.dt_code(x), ops.stream_ptr())
        return buf

    def timestep_embedding(self, t: torch.Tensor) -> torch.Tensor:
        if self._freqs is None:
            self._freqs = self._freqs_cpu.to(t.device)
        B = t.shape[0]
        out = torch.empty((B, self.model_channels), dtype=torch.float32, device=t.device)
        ops.call("rdeic_timestep_embedding", t.data_ptr(), self._freqs.data_ptr(), B, self.model_channels,
                 out.data_ptr(), ops.stream_ptr())
        return out

    def forward(self, x: torch.Tensor, hint: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        # the UNet / control convs need no batch invariance: let small-M, large-K layers split K
        with ops.splitk_allowed():
            return self._forward(x, hint, t, ctx)

    def forward_unconditional(self, x: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        """NoiseEstimator.forward_unconditional (rdeic.py:214-235): the base UNet alone, with its own
        time MLP; no control branch and no zero convs. Used by the spaced sampler's CFG."""
        with ops.splitk_allowed():
            s = self.store
            dt = s.compute_dtype
            t = t.to(device=x.device, dtype=torch.int64).contiguous()
            emb_b = self.base.time_embed(self.timestep_embedding(t))
            ctx = ctx.to(dt).contiguous()
            Bc, Lc, Dc = ctx.shape
            ctx_rows = ctx.view(Bc * Lc, Dc)
            h_base = ops.cast(x, dt)
            hs_base = []
            for lb in self.base.input_blocks:
                h_base = self.base.run_layers(lb, h_base, emb_b, ctx_rows, Bc, Lc)
                hs_base.append(h_base)
            h_base = self.base.run_layers(self.base.middle, h_base, emb_b, ctx_rows, Bc, Lc)
            for lb in self.base.output_blocks:
                h_base = self.base.run_layers(lb, h_base, emb_b, ctx_rows, Bc, Lc, x2=hs_base.pop())
            p = self.base.prefix
            ab = ops.group_norm_ab(h_base, s.get(p + "out.0.weight"), s.get(p + "out.0.bias"), 32, 1e-5)
            return ops.conv2d(h_base, s.conv(p + "out.2"), gn=ab, gn_silu=True, out_f32=True)

    def _forward(self, x: torch.Tensor, hint: torch.Tensor, t: torch.Tensor, ctx: torch.Tensor) -> torch.Tensor:
        """x: fp32 NHWC [B,h,w,4] latent; hint: NHWC [B,h,w,256] (compute dtype);
        t: int64 [B]; ctx: [Bc,77,1024] (compute dtype, Bc in {1, B}). Returns eps fp32 NHWC."""
        s = self.store
        dt = s.compute_dtype
        B = x.shape[0]
        t = t.to(device=x.device, dtype=torch.int64).contiguous()
        temb = self.timestep_embedding(t)
        emb_c = self.ctrl.time_embed(temb)
        emb_b = self.base.time_embed(temb)
        ctx = ctx.to(dt).contiguous()
        Bc, Lc, Dc = ctx.shape
        ctx_rows = ctx.view(Bc * Lc, Dc)
        sc = self.control_scale * self.control_scale  # scale_list * control_scale (rdeic.py:164-165,185)
        h_base = ops.cast(x, dt)
        h_ctr, ctr_x2 = h_base, hint
        hs_base, hs_ctr = [], []
        # GroupNorm statistics travel with the tensors the GroupNorms read: the base features after
        # each zero-conv add (next block, and the decoder's skip concat), the control features, the
        # last decoder block's output (the final norm)
        for i, (lb, lc) in enumerate(zip(self.base.input_blocks, self.ctrl.input_blocks)):
            h_base0 = h_base
            h_base = self.base.run_layers(lb, h_base, emb_b, ctx_rows, Bc, Lc, stats_last=False)
            if i == 0 and dt == torch.bfloat16 and len(lc) == 1 and isinstance(lc[0], Conv) and \
                    h_base0.shape[3] % 64 and hint.shape[3] % 64 == 0:
                # cat(x_t, hint): x_t zero-padded to 64 channels -> both segments take the LDS-DMA path
                h_ctr = ops.conv2d(self._pad64(h_base0), s.conv_split_pad(lc[0].prefix, h_base0.shape[3], 64),
                                   x2=hint, stats=True)
            else:
                h_ctr = self.ctrl.run_layers(lc, h_ctr, emb_c, ctx_rows, Bc, Lc, x2=ctr_x2)
            ctr_x2 = None
            h_base = ops.conv2d(h_ctr, s.conv(self.enc_zero[i], scale=sc), res=h_base, stats=True)
            hs_base.append(h_base)
            hs_ctr.append(h_ctr)
        h_base = self.base.run_layers(self.base.middle, h_base, emb_b, ctx_rows, Bc, Lc, stats_last=False)
        h_ctr = self.ctrl.run_layers(self.ctrl.middle, h_ctr, emb_c, ctx_rows, Bc, Lc, stats_last=False)
        h_base = ops.conv2d(h_ctr, s.conv(self.mid_zero, scale=sc), res=h_base, stats=True)
        nout = len(self.base.output_blocks)
        for i, lb in enumerate(self.base.output_blocks):
            h_base = ops.conv2d(hs_ctr.pop(), s.conv(self.dec_zero[i], scale=sc), res=h_base, stats=True)
            h_base = self.base.run_layers(lb, h_base, emb_b, ctx_rows, Bc, Lc, x2=hs_base.pop(),
                                          stats_last=(i + 1 == nout))
        p = self.base.prefix
        ab = ops.group_norm_ab(h_base, s.get(p + "out.0.weight"), s.get(p + "out.0.bias"), 32, 1e-5)
        return ops.conv2d(h_base, s.conv(p + "out.2"), gn=ab, gn_silu=True, out_f32=True)
