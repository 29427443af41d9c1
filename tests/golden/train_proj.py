"""Seeded random projections of a gradient tensor (shared by the training-step golden generator
and the GPU parity test): 4 float64 dot products with N(0,1) vectors drawn from a CPU generator
seeded by the parameter name, so a permuted or partially wrong gradient cannot match."""
import numpy as np
import torch


def proj_seed(name: str) -> int:
    h = 0
    for b in name.encode():
        h = (h * 131 + b) % 2147483629
    return h


def projections(name: str, g: torch.Tensor) -> np.ndarray:
    gen = torch.Generator().manual_seed(proj_seed(name))
    r = torch.randn((4, g.numel()), generator=gen, dtype=torch.float64)
    return (r @ g.detach().cpu().reshape(-1).double()).numpy()
