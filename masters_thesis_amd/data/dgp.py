"""Synthetic single-factor data-generating process (reference `src/data.py:17-59`).

    r_mkt ~ loc + scale·t_5,  eps ~ t_5(0, 0.314),  alpha ~ N(0.0098, 0.1271),  beta ~ N(0.9444, 0.3521)
    r = alpha + beta·r_mkt + eps          (percent log-returns)

On a GPU the whole (n_stocks, n_samples) matrix is sampled and combined on the device by
``csrc/data.hip`` (two launches; 1e8 Student-t draws in milliseconds instead of the
reference's minutes of CPU ``torch.distributions``).  On the CPU the same distributions are
drawn with a seeded ``torch.Generator``.  Streams are deterministic per ``seed``, not
bit-identical between the two paths.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor


class SyntheticLogReturns:
    """Returns ``(r_stocks (K, N), r_market (N,), alphas (K,), betas (K,))`` from :meth:`generate`."""

    # parameters estimated on the 25 portfolios, outliers removed (reference `src/data.py:34-39`)
    mkt_params = {"loc": 0.0678, "scale": 0.5099, "df": 5}
    idio_params = {"loc": 0.0000, "scale": 0.3140, "df": 5}
    alpha_params = {"loc": 0.0098, "scale": 0.1271}
    beta_params = {"loc": 0.9444, "scale": 0.3521}
    # the reference's alternative "with outliers" estimates (`src/data.py:41-47`), selectable by name
    with_outliers = {
        "mkt_params": {"loc": 0.0538, "scale": 0.6616, "df": 5},
        "idio_params": {"loc": 0.0000, "scale": 0.3539, "df": 5},
        "alpha_params": {"loc": 0.0056, "scale": 0.1501},
        "beta_params": {"loc": 1.0046, "scale": 0.3785},
    }

    @classmethod
    def params(cls, variant: str = "no_outliers"):
        if variant == "with_outliers":
            p = cls.with_outliers
            return p["mkt_params"], p["idio_params"], p["alpha_params"], p["beta_params"]
        if variant != "no_outliers":
            raise ValueError(f"unknown DGP parameter set {variant!r} (no_outliers | with_outliers)")
        return cls.mkt_params, cls.idio_params, cls.alpha_params, cls.beta_params

    @classmethod
    def generate(cls, n_stocks: int, n_samples: int, device=None, seed: Optional[int] = None,
                 variant: str = "no_outliers") -> Tuple[Tensor, Tensor, Tensor, Tensor]:
        from ..ops import dgp as dgp_op

        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        dev = torch.device(device) if device is not None else torch.device("cpu")
        mkt, idio, ap, bp = cls.params(variant)
        return dgp_op.generate(int(n_stocks), int(n_samples), mkt, idio, ap, bp, seed=int(seed), device=dev)
