"""Batched OLS features on the device (reference `src/common.py:132-149`).

Closed-form simple regression per (window, stock) — alpha, beta, unbiased residual
variance and the market's [mean, var] — for all windows in one launch of
``csrc/data.hip::ols_features_kernel`` (one thread per (window, stock)).  CPU tensors use
the PyTorch formulation in ``data/common.py``.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from ..data.common import ols_features as _ols_features_torch
from . import _lib


def ols_features(y: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    if not _lib.use_hip(y) or y.dtype != torch.float32:
        return _ols_features_torch(y)
    y = y.contiguous()
    W, K = y.shape[:2]
    alphas = torch.empty((W, K), device=y.device)
    betas = torch.empty_like(alphas)
    inv_psi = torch.empty_like(alphas)
    factor = torch.empty((W, 2), device=y.device)
    _lib.lib().ols_features(y, alphas, betas, factor, inv_psi)
    return alphas, betas, factor, inv_psi
