"""rdeic_amd — MI355X-native relay-residual-diffusion image codec (RDEIC hot path).

Host code on PyTorch-ROCm (device memory, streams, torch.distributed) drives a C ABI
(include/rdeic_hip.h, librdeic_hip.so) of hand-written gfx950 HIP kernels and host C++
entropy coders. See DESIGN.md.
"""
__version__ = "0.1.0"
