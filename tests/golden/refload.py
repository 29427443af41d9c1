"""Load the reference's own modules (read-only tree at /root/reference) in THIS container, to
produce golden fixtures. Never used on the GPU box and never by the product.

What is stubbed, and why:
  * compressai==1.2.4 and torchac==0.9.3 are absent (no wheels, no network). Their pieces the
    reference calls are provided by oracle/coders_ref.py (our restatement): conv3x3,
    CompressionModel (nn.Module base), GaussianConditional (update/build_indexes/quantize),
    BufferedRansEncoder / RansDecoder, torchac.encode_float_cdf / decode_float_cdf.
  * omegaconf is absent; UNetModel.__init__ only imports ListConfig for an isinstance check.
  * model/rdeic.py imports pyiqa and pytorch_lightning (absent); NoiseEstimator / ControlModule
    / ResBlock / GroupNorm_leq32 / find_denominator / normalization are therefore extracted
    from its AST and executed with the ldm imports it declares.
"""
from __future__ import annotations

import ast
import math
import os
import sys
import types

REF = "/root/reference"


def _install_stubs():
    import torch
    import torch.nn as nn

    from oracle import coders_ref as cr

    if "omegaconf" not in sys.modules:
        om = types.ModuleType("omegaconf")
        lc = types.ModuleType("omegaconf.listconfig")

        class ListConfig(list):
            pass

        lc.ListConfig = ListConfig
        om.listconfig = lc
        sys.modules["omegaconf"] = om
        sys.modules["omegaconf.listconfig"] = lc

    ca = types.ModuleType("compressai")
    layers = types.ModuleType("compressai.layers")
    layers.conv3x3 = lambda i, o, stride=1: nn.Conv2d(i, o, kernel_size=3, stride=stride, padding=1)
    models = types.ModuleType("compressai.models")

    class CompressionModel(nn.Module):
        def __init__(self, *a, **k):
            super().__init__()

        def update(self, scale_table=None, force=False):
            return False

    models.CompressionModel = CompressionModel
    em = types.ModuleType("compressai.entropy_models")

    class EntropyModel(nn.Module):
        pass

    class GaussianConditional(EntropyModel):
        """compressai 1.2.4 semantics (restated in oracle/coders_ref.py)."""

        def __init__(self, scale_table, *a, scale_bound=0.11, tail_mass=1e-9, **k):
            super().__init__()
            self.register_buffer("scale_table", torch.Tensor())
            self.register_buffer("_quantized_cdf", torch.IntTensor())
            self.register_buffer("_offset", torch.IntTensor())
            self.register_buffer("_cdf_length", torch.IntTensor())

        def update_scale_table(self, scale_table, force=False):
            self.scale_table = scale_table.clone().float()
            cdf, lens, off = cr.gaussian_tables(self.scale_table)
            self._quantized_cdf = torch.from_numpy(cdf)
            self._cdf_length = torch.from_numpy(lens)
            self._offset = torch.from_numpy(off)
            return True

        @property
        def quantized_cdf(self):
            return self._quantized_cdf

        @property
        def cdf_length(self):
            return self._cdf_length

        @property
        def offset(self):
            return self._offset

        def build_indexes(self, scales):
            return cr.build_indexes(scales.float(), self.scale_table)

        def quantize(self, inputs, mode, means=None):
            assert mode == "symbols"
            return cr.quantize_symbols(inputs, means)

        def forward(self, inputs, scales, means=None, training=None):
            """Training-mode forward (oracle/train_ref.py restates compressai 1.2.4); the uniform
            noise comes from train_ref.NOISE_QUEUE in call order."""
            from oracle import train_ref
            if training is None:
                training = self.training
            return train_ref.gaussian_forward(inputs, scales, means, training)

    em.EntropyModel = EntropyModel
    em.GaussianConditional = GaussianConditional
    ops = types.ModuleType("compressai.ops")
    ops.quantize_ste = lambda x: (torch.round(x) - x).detach() + x  # compressai/ops/ops.py
    ans = types.ModuleType("compressai.ans")
    ans.BufferedRansEncoder = cr.RansEncoderRef
    ans.RansDecoder = cr.RansDecoderRef
    ca.layers, ca.models, ca.entropy_models, ca.ops, ca.ans = layers, models, em, ops, ans
    for name, mod in [("compressai", ca), ("compressai.layers", layers), ("compressai.models", models),
                      ("compressai.entropy_models", em), ("compressai.ops", ops), ("compressai.ans", ans)]:
        sys.modules[name] = mod

    tac = types.ModuleType("torchac")

    def encode_float_cdf(cdf_float, sym, needs_normalization=True, check_input_bounds=False):
        if check_input_bounds:
            assert cdf_float.min() >= 0 and cdf_float.max() <= 1
            assert sym.max() < cdf_float.shape[-1] - 1
        cdf_int = cr.torchac_int_cdf(cdf_float, needs_normalization)
        rows = cdf_int.reshape(-1, cdf_int.shape[-1]).numpy().view("uint16")
        return cr.ac_encode(rows, sym.reshape(-1).tolist())

    def decode_float_cdf(cdf_float, byte_stream, needs_normalization=True):
        cdf_int = cr.torchac_int_cdf(cdf_float, needs_normalization)
        rows = cdf_int.reshape(-1, cdf_int.shape[-1]).numpy().view("uint16")
        out = cr.ac_decode(rows, byte_stream, rows.shape[0])
        return torch.tensor(out, dtype=torch.int16).reshape(cdf_float.shape[:-1])

    tac.encode_float_cdf = encode_float_cdf
    tac.decode_float_cdf = decode_float_cdf
    sys.modules["torchac"] = tac


_loaded = None


def load():
    """Returns a namespace with the reference classes."""
    global _loaded
    if _loaded is not None:
        return _loaded
    sys.dont_write_bytecode = True
    if REF not in sys.path:
        sys.path.insert(0, REF)
    _install_stubs()
    import torch  # noqa
    from ldm.modules.diffusionmodules import openaimodel, util, model as vae_model
    from ldm.modules import attention
    from ldm import xformers_state
    xformers_state.disable_xformers()
    import model.compression as compression
    import model.ddim_sampler_relay as ddim_mod
    import model.spaced_sampler_relay as spaced_mod
    import utils.ckbd as ckbd

    # AST-extract NoiseEstimator & co. from model/rdeic.py (its module imports pyiqa / PL)
    src = open(os.path.join(REF, "model", "rdeic.py")).read()
    tree = ast.parse(src)
    keep = {"NoiseEstimator", "ControlModule", "ResBlock", "GroupNorm_leq32", "find_denominator", "normalization"}
    body = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef)) and n.name in keep]
    mod = ast.Module(body=body, type_ignores=[])
    ns = dict(torch=torch, th=torch, nn=torch.nn, math=math, conv_nd=util.conv_nd, linear=util.linear,
              zero_module=util.zero_module, timestep_embedding=util.timestep_embedding, checkpoint=util.checkpoint,
              SpatialTransformer=attention.SpatialTransformer, BasicTransformerBlock=attention.BasicTransformerBlock,
              UNetModel=openaimodel.UNetModel, TimestepEmbedSequential=openaimodel.TimestepEmbedSequential,
              ResBlock_orig=openaimodel.ResBlock, Downsample=openaimodel.Downsample,
              Upsample=openaimodel.Upsample, AttentionBlock=openaimodel.AttentionBlock,
              TimestepBlock=openaimodel.TimestepBlock, exists=lambda v: v is not None)
    exec(compile(mod, os.path.join(REF, "model", "rdeic.py"), "exec"), ns)
    _loaded = types.SimpleNamespace(
        UNetModel=openaimodel.UNetModel, NoiseEstimator=ns["NoiseEstimator"], Encoder=vae_model.Encoder,
        Decoder=vae_model.Decoder, ResnetBlock=vae_model.ResnetBlock, AttnBlock=vae_model.AttnBlock,
        SpatialTransformer=attention.SpatialTransformer, UNetResBlock=openaimodel.ResBlock,
        Compression=compression.Compression, DDIMSampler=ddim_mod.DDIMSampler, ckbd=ckbd, util=util,
        SpacedSampler=spaced_mod.SpacedSampler, space_timesteps=spaced_mod.space_timesteps,
        timestep_embedding=util.timestep_embedding)
    return _loaded
