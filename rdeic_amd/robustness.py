"""Bitstream / latent robustness harness (experiments/corruptors.py, experiments/run_robustness.py).

The corruptors are host byte work on ~2.5 KB streams, so they stay on the CPU and consume numpy's
RandomState exactly as the reference does (bit-identical outputs, pinned by
tests/golden/corruptors.npz). The decode side runs the HIP path: each corrupted body is entropy-
decoded on its own (the decode-failure convention of run_robustness.py:277-297 — any exception is a
catastrophic failure with psnr 0 / lpips 1), then every body that decoded goes through one batched
relay-denoise + VAE-decode launch.

Latent corruption draws its randoms from a CPU generator seeded like the reference's
torch.manual_seed(seed) (identical to the reference on CPU tensors; the reference's CUDA-RNG draws
cannot be reproduced on another device, so on-device inputs are corrupted through the CPU copy).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, List, Literal, Optional, Sequence, Tuple

import numpy as np
import torch

from . import bitstream, ops


# ------------------------------------------------------------------ corruptors (corruptors.py)
def bit_flip_bytes(data: bytes, rate: float, seed: int = 42) -> bytes:
    """Flip int(8·len·rate) distinct bits chosen by RandomState(seed).choice (corruptors.py:13-45)."""
    if rate <= 0:
        return data
    rng = np.random.RandomState(seed)
    total_bits = len(data) * 8
    n = int(total_bits * rate)
    if n == 0:
        return data
    pos = rng.choice(total_bits, size=n, replace=False)
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    # distinct positions: one XOR per bit, applied per byte with a scatter of bit masks
    np.bitwise_xor.at(buf, pos // 8, (1 << (pos % 8)).astype(np.uint8))
    return buf.tobytes()


def burst_flip_bytes(data: bytes, burst_rate: float, mean_burst_len: float = 8.0, seed: int = 42) -> bytes:
    """Bursts of geometric length from random starts until int(8·len·rate) distinct bits are
    flipped (corruptors.py:48-95); the RNG call order (randint, geometric) is the reference's."""
    if burst_rate <= 0:
        return data
    rng = np.random.RandomState(seed)
    total_bits = len(data) * 8
    target = int(total_bits * burst_rate)
    if target == 0:
        return data
    flipped = set()
    while len(flipped) < target:
        start = rng.randint(0, total_bits)
        blen = rng.geometric(1.0 / mean_burst_len)
        for off in range(blen):
            flipped.add((start + off) % total_bits)
            if len(flipped) >= target:
                break
    buf = np.frombuffer(data, dtype=np.uint8).copy()
    pos = np.fromiter(flipped, dtype=np.int64, count=len(flipped))
    np.bitwise_xor.at(buf, pos // 8, (1 << (pos % 8)).astype(np.uint8))
    return buf.tobytes()


def latent_corrupt(c_latent: torch.Tensor, mode: Literal["mask_replace", "additive"], rate: float, seed: int = 42,
                   valid_range: Tuple[float, float] = (-3.0, 3.0)) -> torch.Tensor:
    """corruptors.py:98-142. Randoms from a CPU generator seeded `seed` (== torch.manual_seed on CPU)."""
    if rate <= 0:
        return c_latent.clone()
    g = torch.Generator().manual_seed(seed)
    x = c_latent.detach().to("cpu", torch.float32)
    if mode == "mask_replace":
        mask = torch.rand(x.shape, generator=g) < rate
        repl = torch.rand(x.shape, generator=g) * (valid_range[1] - valid_range[0]) + valid_range[0]
        out = x.clone()
        out[mask] = repl[mask]
    elif mode == "additive":
        out = (x + torch.randn(x.shape, generator=g) * rate).clamp(valid_range[0], valid_range[1])
    else:
        raise ValueError(f"Unknown corruption mode: {mode}")
    return out.to(c_latent.device, c_latent.dtype)


def corrupt_bitstream_file(input_path: str, output_path: str, error_type: Literal["random", "burst"], rate: float,
                           seed: int = 42, mean_burst_len: float = 8.0) -> None:
    """corruptors.py:145-176."""
    with open(input_path, "rb") as f:
        data = f.read()
    with open(output_path, "wb") as f:
        f.write(Corruptor("bitstream", error_type, rate, seed, mean_burst_len).corrupt_bytes(data))


def estimate_latent_range(c_latent: torch.Tensor, margin: float = 0.5) -> Tuple[float, float]:
    """corruptors.py:179-194."""
    return c_latent.min().item() - margin, c_latent.max().item() + margin


@dataclass
class Corruptor:
    """corruptors.py:198-241 unified interface."""
    error_space: str
    error_type: str
    rate: float
    seed: int = 42
    mean_burst_len: float = 8.0
    valid_range: Tuple[float, float] = (-3.0, 3.0)

    def corrupt_bytes(self, data: bytes) -> bytes:
        if self.error_space != "bitstream":
            raise ValueError("corrupt_bytes only works with bitstream error_space")
        if self.error_type == "random":
            return bit_flip_bytes(data, self.rate, self.seed)
        if self.error_type == "burst":
            return burst_flip_bytes(data, self.rate, self.mean_burst_len, self.seed)
        raise ValueError(f"Invalid error_type for bitstream: {self.error_type}")

    def corrupt_latent(self, c_latent: torch.Tensor) -> torch.Tensor:
        if self.error_space != "latent":
            raise ValueError("corrupt_latent only works with latent error_space")
        if self.error_type not in ("mask_replace", "additive"):
            raise ValueError(f"Invalid error_type for latent: {self.error_type}")
        return latent_corrupt(c_latent, self.error_type, self.rate, self.seed, self.valid_range)


# ------------------------------------------------------------------ harness (run_robustness.py)
def psnr_u8(a: np.ndarray, b: np.ndarray) -> float:
    mse = float(np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2))
    return float("inf") if mse == 0 else 10.0 * np.log10(255.0 ** 2 / mse)


def try_decompress(model, body: bytes, expect_shape: Optional[Tuple[int, int]] = None):
    """One body through the entropy decoder. Returns (c_latent, guide_hint) NHWC or the exception
    (the reference's `except Exception` → decode_failed, run_robustness.py:277-297). A header whose
    latent shape differs from `expect_shape` is a failure too (the reconstruction could not be
    compared with the original)."""
    try:
        _, shape = bitstream.unpack_body(body)
        if expect_shape is not None and tuple(shape) != tuple(expect_shape):
            raise ValueError(f"corrupted header: latent shape {tuple(shape)} != {tuple(expect_shape)}")
        return model.decompress_bodies([body])
    except Exception as e:  # noqa: BLE001 — the reference's convention
        return e


@torch.no_grad()
def run_bitstream_robustness(model, img_u8: torch.Tensor, context: torch.Tensor, error_type: str,
                             rates: Sequence[float], seeds: Sequence[int], steps: int = 2, sampler: str = "ddim",
                             noise_seed: int = 231, image_ids: Optional[Sequence[str]] = None,
                             mean_burst_len: float = 8.0) -> List[Dict]:
    """Encode each image once, corrupt its bitstream per (rate, seed), decode every corrupted body,
    relay-decode all survivors in one batch, and score PSNR against the original pixels. Returns
    one record per (image, rate, seed) with the reference's columns: PSNR, and SSIM / MS-SSIM on
    the device (rdeic_amd/metrics.py; images of at least 176 pixels a side) — lpips stays None (it
    needs AlexNet weights, not available offline)."""
    B, H, W, _ = img_u8.shape
    ids = list(image_ids) if image_ids is not None else [f"img{i}" for i in range(B)]
    bodies = model.compress_images(img_u8)
    ref = img_u8.cpu().numpy()
    shape0 = bitstream.unpack_body(bodies[0])[1]
    jobs, lat, hint = [], [], []
    for i in range(B):
        bpp = 8.0 * len(bodies[i]) / (H * W)  # 8 * filesize / (H * W) (rdeic.py:667-669)
        for rate in rates:
            for seed in seeds:
                body = Corruptor("bitstream", error_type, rate, seed, mean_burst_len).corrupt_bytes(bodies[i])
                r = try_decompress(model, body, shape0)
                rec = {"image_id": ids[i], "error_space": "bitstream", "error_type": error_type,
                       "error_rate": rate * 100, "seed": seed, "bpp": bpp, "psnr": 0.0, "ssim": None,
                       "ms_ssim": None, "lpips": None, "decode_failed": isinstance(r, Exception)}
                if rec["decode_failed"]:  # the reference's failure row (run_robustness.py:280-295)
                    rec.update(ssim=0.0, ms_ssim=0.0, lpips=1.0, error=f"{type(r).__name__}: {r}")
                else:
                    lat.append(r[0])
                    hint.append(r[1])
                jobs.append((i, rec))
    ok = [(i, rec) for i, rec in jobs if not rec["decode_failed"]]
    if ok:
        c_lat, gh = torch.cat(lat), torch.cat(hint)
        gen = torch.Generator().manual_seed(noise_seed)
        n = c_lat.shape[0]
        noise = ops.nchw_to_nhwc(torch.randn((n, 4, c_lat.shape[1], c_lat.shape[2]), generator=gen).to(c_lat.device),
                                 torch.float32)
        step_noise = None
        if sampler == "ddpm":
            step_noise = torch.stack([ops.nchw_to_nhwc(torch.randn((n, 4, c_lat.shape[1], c_lat.shape[2]),
                                                                   generator=gen).to(c_lat.device), torch.float32)
                                      for _ in range(steps)])
        out_d = model.relay_decode_u8(c_lat, gh, context, noise, steps, sampler, step_noise)
        out = out_d.cpu().numpy()
        tgt = img_u8.to(out_d.device)[torch.tensor([i for i, _ in ok], device=out_d.device)]
        ssim, ms_ssim = (None, None)
        if min(H, W) >= 176:  # 5 MS-SSIM scales need >= 11 pixels at the coarsest one
            from .metrics import ssim_ms_ssim
            ssim, ms_ssim = ssim_ms_ssim(out_d, tgt)
        for k, (i, rec) in enumerate(ok):
            rec["psnr"] = psnr_u8(out[k], ref[i])
            if ssim is not None:
                rec["ssim"], rec["ms_ssim"] = float(ssim[k]), float(ms_ssim[k])
    return [rec for _, rec in jobs]


def write_csv(records: Sequence[Dict], path: str) -> None:
    """results CSV with the reference's column order (run_robustness.py:330-370)."""
    import csv
    cols = ["image_id", "error_space", "error_type", "error_rate", "seed", "bpp", "psnr", "ssim", "ms_ssim", "lpips",
            "decode_failed"]
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols, extrasaction="ignore")
        w.writeheader()
        for r in records:
            w.writerow(r)
