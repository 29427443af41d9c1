"""Full-reference image quality of reconstructions on the device (rdeic_image_ssim, image_mse):
PSNR, SSIM and MS-SSIM as the reference's evaluation scripts report them
(experiments/run_robustness.py:40-93, inference_partition.py:28-70 via pyiqa "psnr" / "ssim" /
"ms_ssim" with test_y_channel). pyiqa is not in this image: SSIM / MS-SSIM follow the published
definition (Wang et al. 2004; Wang, Simoncelli, Bovik 2003) with pyiqa's defaults — YIQ luma,
11x11 Gaussian sigma 1.5, 'valid' windows, relu'd contrast-structure term, 5 scales — and are
checked against the CPU restatement in oracle/metrics_ref.py; parity with pyiqa itself is unpinned.
LPIPS needs an AlexNet backbone that is not available offline (out of scope)."""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from . import _lib, ops

MS_SSIM_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def psnr(pred_u8: torch.Tensor, target_u8: torch.Tensor) -> np.ndarray:
    """Per-image PSNR in dB of uint8 [N,H,W,3] device tensors (10 log10(255^2 / MSE))."""
    n = pred_u8.shape[0]
    mse = torch.empty(n, dtype=torch.float32, device=pred_u8.device)
    ops.call("rdeic_image_mse", target_u8.contiguous().data_ptr(), pred_u8.contiguous().data_ptr(), n,
             pred_u8[0].numel(), mse.data_ptr(), ops.stream_ptr())
    m = mse.cpu().numpy().astype(np.float64)
    with np.errstate(divide="ignore"):
        return np.where(m > 0, 10.0 * np.log10(255.0 ** 2 / np.maximum(m, 1e-30)), 100.0)


def ssim_levels(pred_u8: torch.Tensor, target_u8: torch.Tensor, levels: int = 5) -> np.ndarray:
    """[N, levels, 2] (mean SSIM, mean cs) per scale, on the device."""
    if pred_u8.shape != target_u8.shape or pred_u8.dim() != 4 or pred_u8.shape[3] != 3:
        raise ValueError("expected matching uint8 [N, H, W, 3] images")
    n, h, w, _ = pred_u8.shape
    nf = int(_lib.load().rdeic_image_ssim_ws_floats(n, h, w, levels))
    ws = torch.empty(nf, dtype=torch.float32, device=pred_u8.device)
    out = torch.empty((n, levels, 2), dtype=torch.float32, device=pred_u8.device)
    ops.call("rdeic_image_ssim", pred_u8.contiguous().data_ptr(), target_u8.contiguous().data_ptr(), n, h, w, levels,
             ws.data_ptr(), nf, out.data_ptr(), ops.stream_ptr())
    return out.cpu().numpy().astype(np.float64)


def ssim_ms_ssim(pred_u8: torch.Tensor, target_u8: torch.Tensor) -> Tuple[np.ndarray, np.ndarray]:
    """(SSIM [N], MS-SSIM [N]) of uint8 [N,H,W,3] device images (H, W >= 176 for 5 scales)."""
    lv = ssim_levels(pred_u8, target_u8, len(MS_SSIM_WEIGHTS))
    w = np.asarray(MS_SSIM_WEIGHTS)
    ms = np.prod(lv[:, :-1, 1] ** w[:-1], axis=1) * lv[:, -1, 0] ** w[-1]
    return lv[:, 0, 0], ms
