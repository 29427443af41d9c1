"""Parameter store: reference-named fp32 master tensors on the device + packed MFMA weights.

Names are the reference RDEIC state_dict keys (model.diffusion_model.*, control_model.*,
first_stage_model.*, preprocess_model.*), so a reference checkpoint loads unchanged
(load_state_dict) and the synthetic generator (rdeic_amd/weights.py) is keyed identically.
Packing (rdeic_pack_conv_weight) runs on device once per layer and is cached.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional, Sequence, Tuple

import torch

from . import ops
from . import weights as W


class ParamStore:
    def __init__(self, compute_dtype=torch.bfloat16, device="cuda"):
        self.compute_dtype = compute_dtype
        self.device = torch.device(device)
        self.shapes: Dict[str, Tuple[int, ...]] = {}
        self.t: Dict[str, torch.Tensor] = {}
        self._packed: Dict[tuple, ops.ConvParams] = {}

    # ------------------------------------------------------------ declaration
    def declare(self, name: str, shape: Sequence[int]):
        shape = tuple(int(s) for s in shape)
        if name in self.shapes and self.shapes[name] != shape:
            raise ValueError(f"{name} declared twice with different shapes")
        self.shapes[name] = shape

    def declare_conv(self, prefix: str, cout: int, cin: int, k: int, bias: bool = True):
        self.declare(prefix + ".weight", (cout, cin, k, k))
        if bias:
            self.declare(prefix + ".bias", (cout,))

    def declare_linear(self, prefix: str, cout: int, cin: int, bias: bool = True):
        self.declare(prefix + ".weight", (cout, cin))
        if bias:
            self.declare(prefix + ".bias", (cout,))

    def declare_norm(self, prefix: str, c: int):
        self.declare(prefix + ".weight", (c,))
        self.declare(prefix + ".bias", (c,))

    # ------------------------------------------------------------ materialisation
    def init_synthetic(self, global_seed: int = W.GLOBAL_SEED, rate_gain: float = 1.0):
        """Counter-based synthetic weights generated on device (bit-identical to the oracle's)."""
        for name, shape in self.shapes.items():
            scale, offset = W.init_spec(name, shape, rate_gain)
            t = torch.empty(shape, dtype=torch.float32, device=self.device)
            ops.fill_uniform(t, W.param_seed(name, global_seed), scale, offset)
            self.t[name] = t
        self._packed.clear()

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        missing = [n for n in self.shapes if n not in sd]
        if strict and missing:
            raise KeyError(f"missing parameters: {missing[:8]}{' ...' if len(missing) > 8 else ''}")
        for name, shape in self.shapes.items():
            if name not in sd:
                continue
            v = sd[name]
            if tuple(v.shape) != shape:
                raise ValueError(f"{name}: checkpoint shape {tuple(v.shape)} != {shape}")
            self.t[name] = v.detach().to(device=self.device, dtype=torch.float32).contiguous()
        self._packed.clear()

    def names(self) -> Iterable[str]:
        return self.shapes.keys()

    def get(self, name: str) -> torch.Tensor:
        return self.t[name]

    def has(self, name: str) -> bool:
        return name in self.shapes

    # ------------------------------------------------------------ packed weights
    def conv(self, prefix: str, stride: int = 1, pad: Optional[int] = None, dtype=None,
             scale: float = 1.0, cin_pad: Optional[int] = None, cout_pad: Optional[int] = None) -> ops.ConvParams:
        """Packed conv / linear weights. cin_pad / cout_pad zero-extend the input / output channels
        (zero weight columns / rows and bias): a zero-padded activation keeps 16-byte gathers and
        64-channel blocks; the padded output channels are exactly act(0) = 0 for GELU / leaky / none."""
        dtype = dtype or self.compute_dtype
        key = (prefix, stride, pad, dtype, scale, cin_pad, cout_pad)
        p = self._packed.get(key)
        if p is None:
            w = self.t[prefix + ".weight"]
            b = self.t.get(prefix + ".bias")
            if scale != 1.0:
                w, b = w * scale, (None if b is None else b * scale)
            if cin_pad is not None and cin_pad > w.shape[1]:
                w = torch.nn.functional.pad(w, (0, 0) * (w.dim() - 2) + (0, cin_pad - w.shape[1]))
            if cout_pad is not None and cout_pad > w.shape[0]:
                w = torch.nn.functional.pad(w, (0, 0) * (w.dim() - 1) + (0, cout_pad - w.shape[0]))
                if b is not None:
                    b = torch.nn.functional.pad(b, (0, cout_pad - b.shape[0]))
            k = w.shape[-1] if w.dim() == 4 else 1
            p = ops.ConvParams.pack(w, b, stride=stride, pad=(k // 2 if pad is None else pad), dtype=dtype)
            self._packed[key] = p
        return p

    def conv_split_pad(self, prefix: str, c0: int, c0_pad: int, dtype=None) -> ops.ConvParams:
        """A conv over cat(x [c0 ch], x2) packed for x zero-padded to c0_pad channels: input channels
        [0, c0) stay, [c0, cin) move to [c0_pad, ...), the columns between are zero. Used for the
        control branch's cat(x_t [4], hint [256]) input conv so both segments are 64-channel aligned
        (LDS-DMA path) instead of the 260-channel register-staged path."""
        dtype = dtype or self.compute_dtype
        key = (prefix, "split_pad", c0, c0_pad, dtype)
        p = self._packed.get(key)
        if p is None:
            w = self.t[prefix + ".weight"]
            cout, cin, kh, kw = w.shape
            wp = torch.zeros((cout, cin - c0 + c0_pad, kh, kw), dtype=w.dtype, device=w.device)
            wp[:, :c0] = w[:, :c0]
            wp[:, c0_pad:] = w[:, c0:]
            p = ops.ConvParams.pack(wp, self.t.get(prefix + ".bias"), stride=1, pad=kh // 2, dtype=dtype)
            self._packed[key] = p
        return p

    def conv_geglu(self, prefix: str, dtype=None) -> ops.ConvParams:
        """GEGLU projection (attention.py:49-56, value = rows [0, c), gate = rows [c, 2c)) packed for the
        fused epilogue (ops.linear(geglu=True)): rows reordered in groups of 4 as (value 4j..4j+3,
        gate 4j..4j+3), so one 8-wide output chunk holds matching value / gate channels."""
        dtype = dtype or self.compute_dtype
        key = (prefix, "geglu", dtype)
        p = self._packed.get(key)
        if p is None:
            w = self.t[prefix + ".weight"]
            b = self.t.get(prefix + ".bias")
            c = w.shape[0] // 2
            if c % 4:
                raise ValueError("GEGLU width must be a multiple of 4")
            perm = torch.arange(2 * c, device=w.device).view(2, c // 4, 4).permute(1, 0, 2).reshape(-1)
            p = ops.ConvParams.pack(w[perm], None if b is None else b[perm], dtype=dtype)
            self._packed[key] = p
        return p

    def conv_ln(self, prefixes: Sequence[str], ln_prefix: str, geglu: bool = False, dtype=None) -> ops.ConvParams:
        """Linear(s) fed by LayerNorm(ln_prefix) with the LayerNorm folded in (ops.linear(ln_rows=...)):
        LN(x) W^T + b = rstd (x W'^T - mean colsum(W')) + (b + W beta), W' = W diag(gamma). The packed
        weight is W' (stacked along cout for several prefixes, or GEGLU-interleaved as conv_geglu);
        ln_cs holds the column sums of the PACKED bf16 W' (so the mean term cancels what the GEMM
        accumulated), summed in fp64."""
        dtype = dtype or self.compute_dtype
        key = (tuple(prefixes), "ln", ln_prefix, geglu, dtype)
        p = self._packed.get(key)
        if p is None:
            gamma, beta = self.t[ln_prefix + ".weight"], self.t[ln_prefix + ".bias"]
            ws, bs = [], []
            for pre in prefixes:
                w = self.t[pre + ".weight"]
                b = self.t.get(pre + ".bias")
                ws.append(w)
                bs.append(b if b is not None else torch.zeros(w.shape[0], device=self.device))
            w = torch.cat(ws, 0)
            b = torch.cat(bs, 0).double() + w.double() @ beta.double()
            w = w * gamma[None, :]
            if geglu:
                c = w.shape[0] // 2
                perm = torch.arange(2 * c, device=w.device).view(2, c // 4, 4).permute(1, 0, 2).reshape(-1)
                w, b = w[perm], b[perm]
            p = ops.ConvParams.pack(w, b.float(), dtype=dtype)
            p.ln_cs = p.weight.double().sum(1).float().contiguous()
            self._packed[key] = p
        return p

    def conv_cat(self, prefixes: Sequence[str], dtype=None) -> ops.ConvParams:
        """Several layers with the same input stacked along cout (one GEMM: q|k|v, k|v, emb_layers)."""
        dtype = dtype or self.compute_dtype
        key = (tuple(prefixes), "cat", dtype)
        p = self._packed.get(key)
        if p is None:
            ws, bs = [], []
            for pre in prefixes:
                w = self.t[pre + ".weight"]
                ws.append(w if w.dim() == 4 else w[:, :, None, None])
                b = self.t.get(pre + ".bias")
                bs.append(b if b is not None else torch.zeros(w.shape[0], device=self.device))
            any_bias = any(self.t.get(pre + ".bias") is not None for pre in prefixes)
            w = torch.cat(ws, 0)
            p = ops.ConvParams.pack(w, torch.cat(bs, 0) if any_bias else None, stride=1, pad=w.shape[-1] // 2,
                                    dtype=dtype)
            self._packed[key] = p
        return p
