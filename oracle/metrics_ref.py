"""ORACLE / TEST INFRASTRUCTURE: CPU restatement of the image-quality metrics the reference's
evaluation reports through pyiqa (experiments/run_robustness.py:40-93, baseline_inference.py:37-80,
inference_partition.py:28-70): "psnr", "ssim", "ms_ssim" with pyiqa's defaults (test_y_channel on
YIQ luma rounded to integers, data range 255, 11x11 Gaussian window sigma 1.5 in 'valid' mode,
C1 = (0.01 L)^2, C2 = (0.03 L)^2, relu'd contrast-structure term, MS-SSIM weights
(0.0448, 0.2856, 0.3001, 0.2363, 0.1333) with 2x2 average pooling between the 5 scales and the
product form). pyiqa is not installed in this image (nor is its source in the reference tree), so
this follows the published algorithms (Wang et al. 2004, 2003) — parity with pyiqa is unpinned.
Float64 throughout; the 2D window is applied as the full 11x11 product kernel."""
import numpy as np

WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def y_channel(img_u8: np.ndarray) -> np.ndarray:
    """uint8 HWC RGB -> YIQ luma * 255, rounded half-to-even (pyiqa to_y_channel(img, 255, 'yiq'))."""
    x = img_u8.astype(np.float64) / 255.0
    y = x[..., 0] * 0.299 + x[..., 1] * 0.587 + x[..., 2] * 0.114
    return np.rint(y * 255.0)


def gaussian_2d(size: int = 11, sigma: float = 1.5) -> np.ndarray:
    """fspecial('gaussian'): exp(-(x^2 + y^2) / (2 sigma^2)), normalised to sum 1."""
    r = np.arange(size) - size // 2
    g = np.exp(-(r[:, None] ** 2 + r[None, :] ** 2) / (2.0 * sigma * sigma))
    return g / g.sum()


def filter_valid(x: np.ndarray, win: np.ndarray) -> np.ndarray:
    k = win.shape[0]
    h, w = x.shape
    out = np.zeros((h - k + 1, w - k + 1))
    for dy in range(k):
        for dx in range(k):
            out += win[dy, dx] * x[dy:dy + h - k + 1, dx:dx + w - k + 1]
    return out


def ssim_cs(a: np.ndarray, b: np.ndarray, data_range: float = 255.0):
    """(mean ssim, mean cs) of two luma planes."""
    win = gaussian_2d()
    c1, c2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    mu1, mu2 = filter_valid(a, win), filter_valid(b, win)
    s11 = filter_valid(a * a, win) - mu1 * mu1
    s22 = filter_valid(b * b, win) - mu2 * mu2
    s12 = filter_valid(a * b, win) - mu1 * mu2
    cs = np.maximum((2 * s12 + c2) / (s11 + s22 + c2), 0.0)
    ssim = (2 * mu1 * mu2 + c1) / (mu1 * mu1 + mu2 * mu2 + c1) * cs
    return float(ssim.mean()), float(cs.mean())


def avg_pool2(x: np.ndarray) -> np.ndarray:
    h, w = x.shape
    return x[:h // 2 * 2, :w // 2 * 2].reshape(h // 2, 2, w // 2, 2).mean(axis=(1, 3))


def ssim_ms_ssim(pred_u8: np.ndarray, target_u8: np.ndarray):
    """(SSIM, MS-SSIM) of one uint8 HWC RGB pair."""
    a, b = y_channel(pred_u8), y_channel(target_u8)
    ssim0 = None
    mcs = []
    for lvl in range(len(WEIGHTS)):
        s, c = ssim_cs(a, b)
        if lvl == 0:
            ssim0 = s
        mcs.append(c)
        if lvl + 1 < len(WEIGHTS):
            a, b = avg_pool2(a), avg_pool2(b)
    ms = float(np.prod([mcs[i] ** WEIGHTS[i] for i in range(len(WEIGHTS) - 1)]) * s ** WEIGHTS[-1])
    return ssim0, ms


def psnr(pred_u8: np.ndarray, target_u8: np.ndarray) -> float:
    mse = float(np.mean((pred_u8.astype(np.float64) - target_u8.astype(np.float64)) ** 2))
    return 100.0 if mse == 0 else 10.0 * np.log10(255.0 ** 2 / mse)
