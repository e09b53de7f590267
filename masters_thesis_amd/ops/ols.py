"""Batched OLS features on the device (reference `src/common.py:132-149`).

Closed-form simple regression per (window, stock) — alpha, beta, unbiased residual
variance and the market's [mean, var] — computed for all windows at once on the GPU.
"""
from __future__ import annotations

from typing import Tuple

from torch import Tensor

from ..data.common import ols_features as _ols_features_torch


def ols_features(y: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    return _ols_features_torch(y)
