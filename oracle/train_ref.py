"""TEST INFRASTRUCTURE (oracle): restatement of the compressai 1.2.4 training-mode pieces the
reference's adapter fine-tune step calls, for the golden-vector generator
(tests/golden/make_train_golden.py, which runs the reference's own Compression / VectorQuantiser /
NoiseEstimator / UNetModel modules with these stubbed in) and for the CPU tests.

compressai is absent from /root/reference and from this image (pinned by the reference's
requirements.txt:2 as compressai==1.2.4). Restated from its published source:
  * compressai/ops/bound_ops.py  LowerBoundFunction: forward max(x, bound); backward passes the
    gradient where x >= bound OR the incoming gradient is negative.
  * compressai/entropy_models/entropy_models.py
      EntropyModel.quantize(mode="noise"): inputs + U(-0.5, 0.5) noise (means unused);
      mode="dequantize": round(inputs - means) + means.
      GaussianConditional._standardized_cumulative(x) = 0.5 * erfc(-(2 ** -0.5) * x)
      GaussianConditional._likelihood: v = |inputs - means|, s = LowerBound(0.11)(scales),
        upper - lower of the standardized cumulative at (0.5 - v) / s and (-0.5 - v) / s.
      GaussianConditional.forward(inputs, scales, means, training): quantize ("noise" when
        training else "dequantize"), _likelihood, then LowerBound(1e-9) on the likelihood.
  * compressai/ops/ops.py quantize_ste(x) = (round(x) - x).detach() + x.
The uniform noise is drawn by the caller (NOISE_QUEUE) so the HIP path can consume the same draws.
Never imported by the product (rdeic_amd/)."""
from __future__ import annotations

from typing import List

import torch

SCALE_BOUND = 0.11
LIKELIHOOD_BOUND = 1e-9

# uniform noise tensors consumed in call order by GaussianConditionalTrain.forward(training=True)
NOISE_QUEUE: List[torch.Tensor] = []


class LowerBoundFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bound):
        ctx.save_for_backward(x, bound)
        return torch.max(x, bound)

    @staticmethod
    def backward(ctx, grad_output):
        x, bound = ctx.saved_tensors
        pass_through = (x >= bound) | (grad_output < 0)
        return pass_through * grad_output, None


def lower_bound(x: torch.Tensor, bound: float) -> torch.Tensor:
    return LowerBoundFunction.apply(x, torch.tensor([float(bound)], dtype=x.dtype, device=x.device))


def standardized_cumulative(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * torch.erfc(float(-(2 ** -0.5)) * x)


def likelihood(inputs: torch.Tensor, scales: torch.Tensor, means: torch.Tensor) -> torch.Tensor:
    values = inputs - means
    scales = lower_bound(scales, SCALE_BOUND)
    values = torch.abs(values)
    upper = standardized_cumulative((0.5 - values) / scales)
    lower = standardized_cumulative((-0.5 - values) / scales)
    return upper - lower


def gaussian_forward(inputs, scales, means, training: bool, noise=None):
    """GaussianConditional.forward (outputs, likelihood)."""
    if training:
        if noise is None:
            noise = NOISE_QUEUE.pop(0)
        outputs = inputs + noise
    else:
        outputs = torch.round(inputs - means) + means
    lik = likelihood(outputs, scales, means)
    return outputs, lower_bound(lik, LIKELIHOOD_BOUND)


def quantize_ste(x: torch.Tensor) -> torch.Tensor:
    return (torch.round(x) - x).detach() + x


def adamw_step(params, grads, exp_avg, exp_avg_sq, step: int, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
               weight_decay: float = 1e-2):
    """torch.optim.AdamW's single-tensor update (torch/optim/adamw.py, defaults of the reference's
    configure_optimizers, model/rdeic.py:763-772), in the same op order."""
    b1, b2 = betas
    for p, g, m, v in zip(params, grads, exp_avg, exp_avg_sq):
        p.mul_(1 - lr * weight_decay)
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        denom = (v.sqrt() / (bc2 ** 0.5)).add_(eps)
        p.addcdiv_(m, denom, value=-(lr / bc1))
