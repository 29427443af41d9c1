"""Adapter fine-tune step (config 5) on the HIP kernels.

The reference's light OOD adaptation (train.py:10-28 + configs/finetune_ood.yaml +
configs/model/rdeic_finetune_ood.yaml): sd_locked, is_refine False, so one step is
  get_input      ddpm.py:777-833 + model/rdeic.py:678-686  (VAE encode_hc under no_grad, the
                 posterior sample x 0.18215 -> x_start, h = c x 0.18215; Compression.forward in
                 training mode -> c_latent, likelihoods, q_likelihoods, emb_loss, guide_hint; bpp)
  forward        rdeic.py:774-786 (t ~ U[0, used_timesteps))
  p_losses       rdeic.py:788-835 (noise + (c_latent - x_start) / lamba, q_sample, apply_model =
                 NoiseEstimator(control + frozen base UNet), eps -> x0, loss_simple, logvar 0;
                 loss = l_guide * loss_simple + l_bpp * (bpp + emb_loss) + l_guide * mse(c_latent, x_start))
  optimizer      configure_optimizers (rdeic.py:763-772): AdamW over control_model + preprocess_model
and, with several ranks, the DDP gradient all-reduce of those ~76.7M parameters (bucketed, started
from the backward as buckets complete: parallel.GradBuckets).

Every op (forward and backward) runs through librdeic_hip.so (rdeic_amd/autograd.py); torch's
autograd engine sequences them, and torch supplies device memory and the latent-sized elementwise
loss glue. The trainable parameters live in ONE flat fp32 buffer (grads in another) so the
all-reduce and the AdamW kernel each see one contiguous span.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import torch

from . import autograd as AG
from . import ops
from .rdeic import RDEIC
from .unet import Conv, Down, ResBlock, SpatialTransformer, Up

TRAINABLE_PREFIXES = ("control_model.", "preprocess_model.")


class FineTuneConfig:
    """configs/model/rdeic_finetune_ood.yaml + configs/finetune_ood.yaml (the values the step uses)."""

    def __init__(self, learning_rate=2e-5, l_guide_weight=3.0, l_bpp_weight=1.0, used_timesteps=300,
                 betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, vq_beta=0.25, vq_decay=0.99, vq_temp=0.07):
        self.learning_rate = learning_rate
        self.l_guide_weight = l_guide_weight
        self.l_bpp_weight = l_bpp_weight
        self.used_timesteps = used_timesteps
        self.betas, self.eps, self.weight_decay = betas, eps, weight_decay
        self.vq_beta, self.vq_decay, self.vq_temp = vq_beta, vq_decay, vq_temp


# Split-K policy of the fine-tune step (A/B switch, bench_train.py --ft-splitk): "short" (default) splits every
# small-M layer with >= 8 k-tiles (ops.splitk_allowed(short_k=True)), "long" only the inference rule's >= 32
# k-tile layers, "off" none (one launch per conv: no partial-sum reduce launches).
FT_SPLITK = "short"


def _ft_splitk_ctx():
    import contextlib
    if FT_SPLITK == "off":
        return contextlib.nullcontext()
    return ops.splitk_allowed(short_k=FT_SPLITK == "short")


class FineTuner:
    """Holds the flat trainable parameters / grads / AdamW state of an RDEIC model and runs steps."""

    def __init__(self, model: RDEIC, cfg: Optional[FineTuneConfig] = None,
                 embed_prob: Optional[torch.Tensor] = None):
        """embed_prob: the VectorQuantiser's codebook-usage EMA buffer
        (`preprocess_model.quantize.embed_prob` of a reference checkpoint or of train.py's own; zeros
        when absent, as a freshly built VectorQuantiser, compression_modules.py:239-241). It sets which
        codes the next step re-initialises (decay = exp(-(embed_prob * N * 10) / (1 - 0.99) - 1e-3),
        compression_modules.py:272-296), so a resumed run must carry it."""
        self.m = model
        self.cfg = cfg or FineTuneConfig(used_timesteps=model.used_timesteps)
        st = model.store
        self.dtype = st.compute_dtype
        dev = st.device
        names = [n for n in st.names() if n.startswith(TRAINABLE_PREFIXES)]
        self.names = names
        total = sum(math.prod(st.shapes[n]) for n in names)
        self.flat = torch.empty(total, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        self.offsets: Dict[str, tuple] = {}
        off = 0
        for n in names:
            shape = st.shapes[n]
            k = math.prod(shape)
            self.flat[off:off + k].copy_(st.t[n].reshape(-1))
            p = self.flat[off:off + k].view(shape)
            p.requires_grad_(True)
            p.grad = self.grad[off:off + k].view(shape)
            p._rdeic_gview = p.grad  # conv / linear backward accumulate here directly (autograd.direct_grad_view)
            st.t[n] = p
            self.offsets[n] = (off, k)
            off += k
        st._packed.clear()  # inference packs of trainable layers would be stale after a step
        AG.PACKS.clear()
        AG.STEP_PACKS.clear()
        cb = model.preprocess_model.codebook_size
        self.embed_prob = torch.zeros(cb, dtype=torch.float32, device=dev)  # VectorQuantiser buffer
        if embed_prob is not None:
            if tuple(embed_prob.shape) != (cb,):
                raise ValueError(f"embed_prob has shape {tuple(embed_prob.shape)}, the codebook has {cb} codes")
            self.embed_prob.copy_(embed_prob.to(torch.float32))
        self.step_count = 0
        self.buckets = None

    def load_optimizer_state(self, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, step: int) -> None:
        """Restore AdamW's moments and step count (train.py's checkpoints) so a resumed run continues
        the interrupted one exactly."""
        for dst, src, name in ((self.exp_avg, exp_avg, "exp_avg"), (self.exp_avg_sq, exp_avg_sq, "exp_avg_sq")):
            if src.numel() != dst.numel():
                raise ValueError(f"optimizer.{name} holds {src.numel()} values, the trainable buffer {dst.numel()}")
            dst.copy_(src.reshape(-1).to(torch.float32))
        self.step_count = int(step)

    def enable_ddp(self, bucket_bytes: int = 32 << 20, group=None):
        """Average gradients over the data-parallel ranks, bucketed and overlapped with the backward
        (parallel.GradBuckets). Every rank must hold identical parameters (same init / checkpoint)."""
        from .parallel import GradBuckets
        params = [(self.m.store.t[n], o, k) for n, (o, k) in self.offsets.items()]
        self.buckets = GradBuckets(self.grad, params, bucket_bytes, group)
        return self.buckets

    # ------------------------------------------------------------------ parameters
    def p(self, name: str) -> torch.Tensor:
        return self.m.store.t[name]

    def num_params(self) -> int:
        return self.flat.numel()

    # ------------------------------------------------------------------ layer helpers
    def conv(self, x, prefix, *, stride=1, pad=None, up2=False, emb=None, res=None, act=AG.NONE, slope=0.0,
             pixel_shuffle=False, out_f32=False):
        w = self.p(prefix + ".weight")
        b = self.m.store.t.get(prefix + ".bias")
        kh = w.shape[2] if w.dim() == 4 else 1
        cfg = AG.ConvCfg(kh, kh, stride, kh // 2 if pad is None else pad, up2, pixel_shuffle, act, slope, out_f32,
                         key=None if w.requires_grad else prefix)
        return AG.conv2d(x, w, b, emb=emb, res=res, cfg=cfg)

    def linear(self, x, prefix, *, res=None, out_f32=False):
        w = self.p(prefix + ".weight")
        b = self.m.store.t.get(prefix + ".bias")
        return AG.linear(x, w, b, res=res, key=None if w.requires_grad else prefix, out_f32=out_f32)

    def gn(self, x, prefix, groups, eps, silu, passthrough=False):
        return AG.group_norm(x, self.p(prefix + ".weight"), self.p(prefix + ".bias"), groups, eps, silu, passthrough)

    def ln(self, x, prefix, passthrough=False):
        return AG.layer_norm(x, self.p(prefix + ".weight"), self.p(prefix + ".bias"), 1e-5, passthrough)

    # ------------------------------------------------------------------ UNet / control (openaimodel.py, rdeic.py)
    def time_embed(self, net, temb):
        """SiLU(time_embed(t_emb)) — the SiLU every emb_layers starts with (openaimodel.py:235-241)."""
        e = AG.act(self.linear(temb, net.prefix + "time_embed.0"), AG.SILU)
        e = self.linear(e, net.prefix + "time_embed.2")
        return AG.act(e, AG.SILU)

    def resblock(self, rb: ResBlock, x, semb):
        """openaimodel.py:254-274 / rdeic.py:566-598 (emb_layers Linear, no scale-shift norm)."""
        # x feeds the first norm and the skip path: the skip path takes the norm's passthrough alias, so its
        # gradient is added inside the norm's backward kernel (no autograd add launch)
        h, xs = self.gn(x, rb.prefix + ".in_layers.0", rb.gn_in, 1e-5, True, passthrough=True)
        emb = self.linear(semb, rb.prefix + ".emb_layers.1")
        h = self.conv(h, rb.prefix + ".in_layers.2", emb=emb)
        h = self.gn(h, rb.prefix + ".out_layers.0", rb.gn_out, 1e-5, True)
        skip = xs if rb.cin == rb.cout else self.conv(xs, rb.prefix + ".skip_connection")
        return self.conv(h, rb.prefix + ".out_layers.3", res=skip)

    def transformer(self, t: SpatialTransformer, x, ctx_rows, batch):
        """SpatialTransformer with use_linear (attention.py:288-350), BasicTransformerBlock (:255-285)."""
        B, H, W_, C = x.shape
        L = H * W_
        tb = t.prefix + ".transformer_blocks.0"
        # every residual input also feeds a norm: the residual takes the norm's passthrough alias (see resblock)
        h, xs = self.gn(x, t.prefix + ".norm", t.gn, 1e-6, False, passthrough=True)
        h = self.linear(h.reshape(B * L, C), t.prefix + ".proj_in")
        scale = t.dh ** -0.5
        n1, hs = self.ln(h, tb + ".norm1", passthrough=True)
        q = self.linear(n1, tb + ".attn1.to_q")
        k = self.linear(n1, tb + ".attn1.to_k")
        v = self.linear(n1, tb + ".attn1.to_v")
        o = AG.attention(q, k, v, batch, t.heads, scale)
        h = self.linear(o, tb + ".attn1.to_out.0", res=hs)
        n2, hs = self.ln(h, tb + ".norm2", passthrough=True)
        q = self.linear(n2, tb + ".attn2.to_q")
        k = self.linear(ctx_rows, tb + ".attn2.to_k")
        v = self.linear(ctx_rows, tb + ".attn2.to_v")
        o = AG.attention(q, k, v, batch, t.heads, scale)
        h = self.linear(o, tb + ".attn2.to_out.0", res=hs)
        n3, hs = self.ln(h, tb + ".norm3", passthrough=True)
        g = AG.geglu(self.linear(n3, tb + ".ff.net.0.proj"))
        h = self.linear(g, tb + ".ff.net.2", res=hs)
        out = self.linear(h, t.prefix + ".proj_out", res=xs.reshape(B * L, C))
        return out.view(B, H, W_, C)

    def run_layers(self, net, layers, x, semb, ctx_rows, batch):
        for layer in layers:
            if isinstance(layer, Conv):
                x = self.conv(x, layer.prefix)
            elif isinstance(layer, ResBlock):
                x = self.resblock(layer, x, semb)
            elif isinstance(layer, SpatialTransformer):
                x = self.transformer(layer, x, ctx_rows, batch)
            elif isinstance(layer, Down):
                x = self.conv(x, layer.prefix, stride=2, pad=1)
            elif isinstance(layer, Up):
                x = self.conv(x, layer.prefix, up2=True)
            else:
                raise TypeError(layer)
        return x

    def noise_estimator(self, x_noisy, hint, t, ctx):
        """NoiseEstimator.forward (rdeic.py:174-212), differentiable. x_noisy fp32 NHWC [B,h,w,4];
        hint NHWC compute dtype [B,h,w,256]; ctx [B,77,1024] (compute dtype); returns eps fp32 NHWC."""
        ne = self.m.control_model
        if ne.control_scale != 1.0:
            raise NotImplementedError("control_scale != 1 in the fine-tune step")
        B = x_noisy.shape[0]
        temb = ne.timestep_embedding(t.to(device=x_noisy.device, dtype=torch.int64).contiguous())
        semb_c = self.time_embed(ne.ctrl, temb)
        semb_b = self.time_embed(ne.base, temb)
        Bc, Lc, Dc = ctx.shape
        if Bc != B:
            ctx = ctx.expand(B, Lc, Dc)
        ctx_rows = ctx.reshape(B * Lc, Dc).to(self.dtype).contiguous()
        h_base = AG.cast(x_noisy, self.dtype)
        h_ctr = torch.cat([h_base, hint], dim=3)
        hs_base, hs_ctr = [], []
        for i, (lb, lc) in enumerate(zip(ne.base.input_blocks, ne.ctrl.input_blocks)):
            h_base = self.run_layers(ne.base, lb, h_base, semb_b, ctx_rows, B)
            h_ctr = self.run_layers(ne.ctrl, lc, h_ctr, semb_c, ctx_rows, B)
            h_base = self.conv(h_ctr, ne.enc_zero[i], res=h_base)
            hs_base.append(h_base)
            hs_ctr.append(h_ctr)
        h_base = self.run_layers(ne.base, ne.base.middle, h_base, semb_b, ctx_rows, B)
        h_ctr = self.run_layers(ne.ctrl, ne.ctrl.middle, h_ctr, semb_c, ctx_rows, B)
        h_base = self.conv(h_ctr, ne.mid_zero, res=h_base)
        for i, lb in enumerate(ne.base.output_blocks):
            h_base = self.conv(hs_ctr.pop(), ne.dec_zero[i], res=h_base)
            h_base = torch.cat([h_base, hs_base.pop()], dim=3)
            h_base = self.run_layers(ne.base, lb, h_base, semb_b, ctx_rows, B)
        p = ne.base.prefix
        h = self.gn(h_base, p + "out.0", 32, 1e-5, True)
        return self.conv(h, p + "out.2", out_f32=True)

    # ------------------------------------------------------------------ Compression.forward (training)
    def _block(self, blk, x):
        pre, kind, ci, co = blk
        L = AG.LEAKY
        if kind == "conv":
            return self.conv(x, pre)
        if kind == "rb":
            identity = x if ci == co else self.conv(x, pre + ".adaptor")
            out = self.conv(x, pre + ".conv1", act=L, slope=0.01)
            return self.conv(out, pre + ".conv2", act=L, slope=0.01, res=identity)
        if kind == "rbs":
            out = self.conv(x, pre + ".conv1", stride=2, pad=1, act=L, slope=0.01)
            identity = self.conv(x, pre + ".downsample", stride=2, pad=0)
            return self.conv(out, pre + ".conv2", act=L, slope=0.1, res=identity)
        if kind == "rbu":
            out = self.conv(x, pre + ".subpel_conv.0", pixel_shuffle=True, act=L, slope=0.01)
            identity = self.conv(x, pre + ".upsample.0", pixel_shuffle=True)
            return self.conv(out, pre + ".conv", act=L, slope=0.1, res=identity)
        raise ValueError(kind)

    def _seq(self, blocks, x):
        for b in blocks:
            x = self._block(b, x)
        return x

    def _ep(self, name, i, x):
        p = self.m.preprocess_model.p
        h = self.conv(x, f"{p}{name}.{i}.fusion.0", act=AG.GELU)
        h = self.conv(h, f"{p}{name}.{i}.fusion.2", act=AG.GELU)
        return self.conv(h, f"{p}{name}.{i}.fusion.4")

    def _channel_ctx(self, i, x):
        p = self.m.preprocess_model.p
        h = self.conv(x, f"{p}channel_context.{i}.fushion.0", act=AG.GELU)
        h = self.conv(h, f"{p}channel_context.{i}.fushion.2", act=AG.GELU)
        return self.conv(h, f"{p}channel_context.{i}.fushion.4")

    def compression_forward(self, h, slice_noise: Sequence[torch.Tensor]):
        """Compression.forward (compression.py:52-149) in training mode. h NHWC compute dtype
        [B,H/8,W/8,512]; slice_noise[i] fp32 NHWC [B,hy,wy,c_i] (the U(-0.5,0.5) draws). Returns
        (c_latent fp32 NHWC, S = sum ln lik (noise), qS (dequantize, no grad), emb_loss[1], guide_hint)."""
        cm = self.m.preprocess_model
        p = cm.p
        y = self._seq(cm.g_a, h)
        z = self._seq(cm.hyper_enc, y)
        zq, emb_loss = AG.VQTrainFn.apply(z, self.p(p + "quantize.embedding.weight"), self.embed_prob,
                                          self.cfg.vq_beta, self.cfg.vq_decay, self.cfg.vq_temp)
        hyper = self._seq(cm.hyper_dec, zq)
        S_tot, qS_tot = None, None
        yhat_slices: List[torch.Tensor] = []
        for i, c in enumerate(cm.slice_ch):
            s0 = cm.slice_off[i]
            ys = y[..., s0:s0 + c]
            if i == 0:
                pa = self._ep("entropy_parameters_anchor", 0, hyper)
                channel_ctx = None
            else:
                channel_ctx = self._channel_ctx(i, torch.cat(yhat_slices, dim=3))
                pa = self._ep("entropy_parameters_anchor", i, torch.cat([channel_ctx, hyper], dim=3))
            anchor_hat = AG.CkbdAnchorFn.apply(ys, pa)
            local_ctx = self.conv(anchor_hat, f"{p}local_context.{i}")
            ctx_in = [local_ctx, hyper] if i == 0 else [local_ctx, channel_ctx, hyper]
            pn = self._ep("entropy_parameters_nonanchor", i, torch.cat(ctx_in, dim=3))
            S, qS, non = AG.CkbdLikFn.apply(ys, pa, pn, slice_noise[i])
            yhat_slices.append(anchor_hat + non)
            S_tot = S if S_tot is None else S_tot + S
            qS_tot = qS if qS_tot is None else qS_tot + qS
        y_hat = torch.cat(yhat_slices, dim=3)
        guide_hint = self._seq(cm.g_s, y_hat)
        c_latent = self.conv(guide_hint, p + "out", out_f32=True)
        return c_latent, S_tot, qS_tot, emb_loss, guide_hint

    # ------------------------------------------------------------------ the step
    @torch.no_grad()
    def get_first_stage(self, img_u8: torch.Tensor, post_eps_nhwc: torch.Tensor):
        """img_u8: uint8 [B,H,W,3] on the device (the batch's 'jpg', x = u8/255*2-1 as inference's
        encode path). Returns (x_start fp32 NHWC, h compute dtype NHWC): the posterior sample
        (mean + std * post_eps, distributions.py:24-37) x scale_factor and c x scale_factor
        (ddpm.py:786-789, encode_first_stage under no_grad)."""
        m = self.m
        B, H, W_, _ = img_u8.shape
        cpad = 8 if self.dtype == torch.bfloat16 else 3
        x = torch.empty((B, H, W_, cpad), dtype=self.dtype, device=img_u8.device)
        ops.call("rdeic_image_u8_to_nhwc", img_u8.contiguous().data_ptr(), B, H, W_, x.data_ptr(), cpad,
                 ops.dt_code(x), ops.stream_ptr())
        h, mom = m.first_stage_model.encode_hc_moments(x, out_mul=m.scale_factor)
        mean, logvar = mom[..., :4], mom[..., 4:]
        std = torch.exp(0.5 * torch.clamp(logvar, -30.0, 20.0))
        x_start = m.scale_factor * (mean + std * post_eps_nhwc)
        return x_start.contiguous(), h

    def losses(self, x_start, h, ctx, t, noise, slice_noise):
        """p_losses (rdeic.py:788-835, non-refine) + the bpp of get_input; returns (loss, loss_dict)."""
        m, cfg = self.m, self.cfg
        c_latent, S, qS, emb_loss, guide_hint = self.compression_forward(h, slice_noise)
        B, hl, wl, _ = x_start.shape
        num_pixels = B * hl * wl * 64
        bpp = AG.bpp_from_sum(S, num_pixels)
        q_bpp = AG.bpp_from_sum(qS, num_pixels)
        lamba = m.sqrt_recipm1_alphas_cumprod[m.used_timesteps - 1]
        t = t.to(device=x_start.device, dtype=torch.int64)
        noise = noise + (c_latent - x_start) / lamba
        a = m.sqrt_alphas_cumprod[t].view(-1, 1, 1, 1)
        b = m.sqrt_one_minus_alphas_cumprod[t].view(-1, 1, 1, 1)
        x_noisy = a * x_start + b * noise
        eps = self.noise_estimator(x_noisy, guide_hint, t, ctx)
        model_output = (m.sqrt_recip_alphas_cumprod[t].view(-1, 1, 1, 1) * x_noisy -
                        m.sqrt_recipm1_alphas_cumprod[t].view(-1, 1, 1, 1) * eps)
        loss_simple = ((x_start - model_output) ** 2).mean(dim=(1, 2, 3))
        loss = cfg.l_guide_weight * loss_simple.mean()  # logvar_t = 0: loss_simple / exp(0) + 0
        loss = loss + cfg.l_bpp_weight * bpp[0]
        loss = loss + cfg.l_bpp_weight * emb_loss[0]
        loss_guide = ((x_start - c_latent) ** 2).mean()
        loss = loss + cfg.l_guide_weight * loss_guide
        d = {"T/l_simple": loss_simple.mean(), "T/l_bpp": bpp[0], "T/q_bpp": q_bpp[0], "T/l_emb": emb_loss[0],
             "T/l_guide": loss_guide, "T/loss": loss}
        # detached: holding the autograd graph past the step would keep the parameters' AccumulateGrad
        # nodes (and their stream) alive into the next step / a graph capture
        self._last = dict(c_latent=c_latent.detach(), eps=eps.detach(), x_noisy=x_noisy.detach(),
                          guide_hint=guide_hint.detach())
        return loss, d

    def zero_grad(self):
        self.grad.zero_()
        for n in self.offsets:  # direct-gradient use counts (autograd.count_direct_use) start at zero
            p = self.m.store.t[n]
            p._rdeic_uses = 0
            p._rdeic_direct = False

    def adam_scalars(self, step: int) -> torch.Tensor:
        """[-lr / (1 - beta1^step), sqrt(1 - beta2^step)] in Python doubles, as torch.optim.AdamW forms them."""
        c = self.cfg
        b1, b2 = c.betas
        return torch.tensor([-c.learning_rate / (1 - b1 ** step), (1 - b2 ** step) ** 0.5], dtype=torch.float32)

    def adamw_launch(self, sc_dev: torch.Tensor):
        c = self.cfg
        AG.call("rdeic_adamw_dev", self.flat.data_ptr(), self.grad.data_ptr(), self.exp_avg.data_ptr(),
                self.exp_avg_sq.data_ptr(), self.flat.numel(), float(c.learning_rate), float(c.betas[0]),
                float(c.betas[1]), float(c.eps), float(c.weight_decay), sc_dev.data_ptr(), ops.stream_ptr())

    def optimizer_step(self):
        """AdamW over the flat trainable buffer (torch.optim.AdamW defaults, lr from the config)."""
        self.step_count += 1
        if getattr(self, "_sc", None) is None:
            self._sc = torch.zeros(2, dtype=torch.float32, device=self.flat.device)
        self._sc.copy_(self.adam_scalars(self.step_count), non_blocking=True)
        self.adamw_launch(self._sc)

    def training_step(self, img_u8, ctx, draws: dict, sync_grads=None):
        """One step: forward, backward, (all-reduce), AdamW. img_u8 uint8 [B,H,W,3] on the device;
        draws: t [B], post_eps / noise fp32 NHWC [B,h,w,4], slice_noise list of fp32 NHWC.
        Returns the loss dict (device scalars)."""
        self.zero_grad()
        AG.STEP_PACKS.refresh()  # the trainable layers' packed weights, one launch (after the last update)
        x_start, h = self.get_first_stage(img_u8, draws["post_eps"])
        if self.buckets is not None:
            self.buckets.begin()
        # training needs no batch invariance anywhere: small-M / large-K convs (B=1 UNet levels, input
        # gradients) may split K (deterministic, fixed-order reduction)
        with _ft_splitk_ctx(), AG.STEP_PACKS.active():
            loss, d = self.losses(x_start, h, ctx, draws["t"], draws["noise"], draws["slice_noise"])
            loss.backward()
        if self.buckets is not None:
            self.buckets.finish()
        elif sync_grads is not None:
            sync_grads(self.grad)
        self.optimizer_step()
        if self.buckets is not None:
            self.sync_codebook()
        return {k: v.detach() for k, v in d.items()}

    def sync_codebook(self, src: int = 0):
        """Data-parallel replicas: VectorQuantiser.forward re-initialises dead codes in place from each
        rank's OWN batch (compression_modules.py:272-296), which no gradient all-reduce covers (the
        reference only ever trains on one GPU, finetune_ood.yaml:28-30). Keep the replicas identical by
        taking rank `src`'s codebook and usage EMA after the step (16 MB broadcast)."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            return
        o, k = self.offsets[self.m.preprocess_model.p + "quantize.embedding.weight"]
        dist.broadcast(self.flat[o:o + k], src)
        dist.broadcast(self.embed_prob, src)


class CapturedStep:
    """The whole single-GPU fine-tune step (zero grads, forward, backward, AdamW) captured ONCE as a
    hipGraph (torch.cuda.CUDAGraph) and replayed per step. At B=1 the eager step is host-bound
    (~1,800 launches, each through torch autograd and ctypes); a replay issues them from the graph.
    Inputs live in static buffers (copied in before each replay); AdamW's step-dependent scalars come
    from a device buffer (rdeic_adamw_dev). Capture runs one eager warm-up step on a side stream
    (packs the frozen layers' weights, sizes the workspaces) and then restores the optimizer state,
    so the first replay is the tuner's next step. Multi-GPU steps stay eager (the bucketed all-reduce
    is launched from the backward's hooks)."""

    def __init__(self, ft: "FineTuner", img_u8: torch.Tensor, ctx: torch.Tensor, draws: dict):
        if ft.buckets is not None:
            raise ValueError("graph capture is single-GPU (the DDP all-reduce runs from backward hooks)")
        self.ft = ft
        self.img = img_u8.clone()
        self.ctx = ctx.clone()
        self.d = {k: (v.clone() if torch.is_tensor(v) else [x.clone() for x in v]) for k, v in draws.items()}
        self.sc = torch.zeros(2, dtype=torch.float32, device=img_u8.device)
        snap = [t.clone() for t in (ft.flat, ft.exp_avg, ft.exp_avg_sq, ft.embed_prob)]
        step0 = ft.step_count
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            ft.training_step(self.img, self.ctx, self.d)          # warm-up (eager)
            AG.STEP_PACKS.refresh()  # builds the pack job table outside the capture
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=side):  # the stream the warm-up ran on
            self.out = self._body()
        for t, v in zip((ft.flat, ft.exp_avg, ft.exp_avg_sq, ft.embed_prob), snap):
            t.copy_(v)
        ft.step_count = step0
        torch.cuda.synchronize()

    def _body(self):
        ft = self.ft
        ft.zero_grad()
        AG.STEP_PACKS.refresh()
        x_start, h = ft.get_first_stage(self.img, self.d["post_eps"])
        with _ft_splitk_ctx(), AG.STEP_PACKS.active():
            loss, d = ft.losses(x_start, h, self.ctx, self.d["t"], self.d["noise"], self.d["slice_noise"])
            loss.backward()
        d = {k: v.detach() for k, v in d.items()}
        del loss
        ft.adamw_launch(self.sc)
        return d

    def step(self, img_u8: torch.Tensor, draws: dict) -> dict:
        ft = self.ft
        self.img.copy_(img_u8, non_blocking=True)
        for k, v in draws.items():
            if torch.is_tensor(v):
                self.d[k].copy_(v, non_blocking=True)
            else:
                for dst, src in zip(self.d[k], v):
                    dst.copy_(src, non_blocking=True)
        ft.step_count += 1
        self.sc.copy_(ft.adam_scalars(ft.step_count), non_blocking=True)
        self.graph.replay()
        return self.out


def nchw_draws_to_nhwc(dr: dict, device) -> dict:
    """train_draws (NCHW, CPU) -> device NHWC fp32 tensors for FineTuner.training_step."""
    f = lambda a: a.permute(0, 2, 3, 1).contiguous().to(device=device, dtype=torch.float32)  # noqa: E731
    return dict(t=dr["t"].to(device), post_eps=f(dr["post_eps"]), noise=f(dr["noise"]),
                slice_noise=[f(s) for s in dr["slice_noise"]])
