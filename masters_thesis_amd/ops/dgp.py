"""Synthetic DGP on the GPU (reference `src/data.py:49-59`).

Draws the market and idiosyncratic Student-t(5) variates and the Normal alpha/beta
directly on the device (1e8 draws in well under a second on MI355X instead of
minutes of host sampling), then combines them with one fused broadcast
``alpha + beta * r_mkt + eps``.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
from torch import Tensor


def _student_t(shape, df: float, loc: float, scale: float, gen: torch.Generator, device) -> Tensor:
    z = torch.randn(shape, generator=gen, device=device)
    # chi2_df / df via Gamma(df/2, 2)
    g = torch._standard_gamma(torch.full(shape, df / 2.0, device=device), generator=gen) * 2.0
    return loc + scale * z * torch.rsqrt(g / df)


def generate(n_stocks: int, n_samples: int, mkt: Dict, idio: Dict, ap: Dict, bp: Dict, *, seed: int = 0,
             device=None) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    dev = torch.device(device)
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed))
    r_market = _student_t((n_samples,), mkt["df"], mkt["loc"], mkt["scale"], gen, dev)
    r_idio = _student_t((n_stocks, n_samples), idio["df"], idio["loc"], idio["scale"], gen, dev)
    alphas = ap["loc"] + ap["scale"] * torch.randn(n_stocks, generator=gen, device=dev)
    betas = bp["loc"] + bp["scale"] * torch.randn(n_stocks, generator=gen, device=dev)
    r_idio.addcmul_(betas.unsqueeze(1), r_market.unsqueeze(0)).add_(alphas.unsqueeze(1))
    return r_idio, r_market, alphas, betas
