"""Synthetic DGP on the GPU (reference `src/data.py:49-59`).

Draws the market and idiosyncratic Student-t variates and the Normal alpha/beta
directly on the device and combines them as ``alpha + beta * r_mkt + eps`` in the same
pass: ``csrc/data.hip`` (counter-hash normals, Student-t = z / sqrt(chi2_df / df) for the
configs' integer df; two launches for the whole matrix).  Non-integer df falls back to
the torch.distributions-style sampler below.
"""
from __future__ import annotations

from typing import Dict, Tuple

import torch
from torch import Tensor

from . import _lib


def _student_t(shape, df: float, loc: float, scale: float, gen: torch.Generator, device) -> Tensor:
    z = torch.randn(shape, generator=gen, device=device)
    # chi2_df / df via Gamma(df/2, 2)
    g = torch._standard_gamma(torch.full(shape, df / 2.0, device=device), generator=gen) * 2.0
    return loc + scale * z * torch.rsqrt(g / df)


def generate(n_stocks: int, n_samples: int, mkt: Dict, idio: Dict, ap: Dict, bp: Dict, *, seed: int = 0,
             device=None) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    dev = torch.device(device)
    dfs = (float(mkt["df"]), float(idio["df"]))
    if _lib.use_hip(torch.empty(0, device=dev)) and all(d.is_integer() and 1 <= d <= 64 for d in dfs):
        r_market = torch.empty(n_samples, device=dev)
        r_stocks = torch.empty((n_stocks, n_samples), device=dev)
        alphas = torch.empty(n_stocks, device=dev)
        betas = torch.empty(n_stocks, device=dev)
        _lib.lib().dgp(int(seed) & ((1 << 63) - 1), int(dfs[0]), float(mkt["loc"]), float(mkt["scale"]),
                       int(dfs[1]), float(idio["loc"]), float(idio["scale"]), float(ap["loc"]),
                       float(ap["scale"]), float(bp["loc"]), float(bp["scale"]), r_market, r_stocks, alphas, betas)
        return r_stocks, r_market, alphas, betas
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed))
    r_market = _student_t((n_samples,), mkt["df"], mkt["loc"], mkt["scale"], gen, dev)
    r_idio = _student_t((n_stocks, n_samples), idio["df"], idio["loc"], idio["scale"], gen, dev)
    alphas = ap["loc"] + ap["scale"] * torch.randn(n_stocks, generator=gen, device=dev)
    betas = bp["loc"] + bp["scale"] * torch.randn(n_stocks, generator=gen, device=dev)
    r_idio.addcmul_(betas.unsqueeze(1), r_market.unsqueeze(0)).add_(alphas.unsqueeze(1))
    return r_idio, r_market, alphas, betas
