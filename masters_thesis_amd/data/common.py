"""Dataset math in plain PyTorch: windowing, features, OLS targets, Woodbury covariance / NLL oracles.

Behaviour follows the reference's `src/common.py` (cited per function).  These are the CPU
implementations and the fp64 oracles the HIP kernels are tested against; the device paths
live in ``ops.ols`` (``csrc/data.hip``) and ``ops.losses`` (``csrc/losses.hip``).

Differences in *how* (not what):

* ``ols`` is the closed-form simple regression instead of ``pinv(XᵀX)·Xᵀy``
  (`src/common.py:33-47`).  For a non-constant regressor the two are the same estimator; for a
  constant regressor (XᵀX rank 1) the min-norm pinv solution is reproduced explicitly.
* ``woodbury_nll_closed_form`` evaluates the reference NLL in O(K·n) without the K×K matrix or
  its LU ``logdet``; ``gaussian_nll_dense`` keeps the dense formulation
  (`src/model.py:44-69`) as the oracle.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
from torch import Tensor

__all__ = ["ols", "inverse_returns_covariance", "gaussian_nll_dense", "woodbury_nll_closed_form",
           "lookback_target_split", "add_quadratic_features", "ols_features", "append_feature"]


def _regress(x: Tensor, y: Tensor) -> Tuple[Tensor, Tensor]:
    """x (B, n), y (B, K, n) -> alpha, beta (B, K) with pinv semantics for a constant x."""
    n = x.shape[-1]
    xm = x.mean(-1, keepdim=True)                       # (B, 1)
    ym = y.mean(-1)                                     # (B, K)
    xc = x - xm
    sxx = (xc * xc).sum(-1, keepdim=True)               # (B, 1)
    sxy = (y * xc.unsqueeze(1)).sum(-1)                 # (B, K)
    # pinv's cutoff drops singular values below 2·eps·σ_max.  XᵀX has σ_max ≈ n(1 + xm²) and
    # σ_min ≈ sxx / (1 + xm²): below that floor the system is treated as rank 1, like pinv.
    eps = torch.finfo(x.dtype).eps
    floor = 2 * eps * n * (1 + xm * xm) ** 2
    degenerate = sxx <= floor
    beta_reg = sxy / torch.where(degenerate, torch.ones_like(sxx), sxx)
    alpha_reg = ym - beta_reg * xm
    # min-norm [a, b] with a + b·x0 = mean(y) for the constant regressor x0
    x0 = xm
    inv = 1.0 / (1.0 + x0 * x0)
    alpha = torch.where(degenerate, ym * inv, alpha_reg)
    beta = torch.where(degenerate, ym * x0 * inv, beta_reg)
    return alpha, beta


def ols(X: Tensor, y: Tensor) -> Tuple[Tensor, Tensor]:
    """Intercept and slope of ``y`` regressed on ``X`` (reference `src/common.py:5-31`).

    X: (n,) or (B, n); y: (K, n) or (B, K, n).  Unbatched inputs return squeezed (K,) results,
    like the reference.
    """
    if X.dim() <= 1 and y.dim() <= 2:
        a, b = _regress(X.unsqueeze(0), y.unsqueeze(0))
        return a.squeeze(), b.squeeze()
    if X.dim() == 1:
        X = X.unsqueeze(0).expand(y.shape[0], -1)
    if y.dim() == 2:
        y = y.unsqueeze(0)
    return _regress(X, y)


def inverse_returns_covariance(beta: Tensor, inv_psi: Tensor, f_var: Tensor) -> Tensor:
    """Dense Σ⁻¹ = Ψ⁻¹ − Ψ⁻¹ββᵀΨ⁻¹ / (1/σ_f² + βᵀΨ⁻¹β) (reference `src/common.py:50-78`).

    beta (K, 1), inv_psi (K, K) diagonal, f_var scalar.  Only the oracle / eager-reference path
    builds this matrix; the fused kernels never do.
    """
    w_beta = inv_psi @ beta                              # (K, 1)
    denom = 1.0 / f_var + (beta.mT @ w_beta)             # (1, 1)
    return inv_psi - (w_beta @ w_beta.mT) / denom


def gaussian_nll_dense(mean: Tensor, inv_cov: Tensor, target: Tensor) -> Tensor:
    """½·(n·(K ln 2π − logdet Σ⁻¹) + tr(Dᵀ Σ⁻¹ D)), D = target − mean (reference `src/model.py:44-69`).

    mean (K, 1) or (K, n), inv_cov (K, K), target (K, n).  Not divided by n.
    """
    K, n = target.shape[-2], target.shape[-1]
    D = target - mean
    quad = (D * (inv_cov @ D)).sum()
    logdet = torch.logdet(inv_cov)
    return 0.5 * (n * (K * math.log(2 * math.pi) - logdet) + quad)


def woodbury_nll_closed_form(alpha: Tensor, beta: Tensor, f_mean: Tensor, f_var: Tensor, w: Tensor,
                             r: Tensor) -> Tensor:
    """The same NLL in O(K·n): matrix determinant lemma + Woodbury quadratic form.

    alpha, beta, w = diag(Ψ⁻¹): (K,); r: (K, n).
    """
    K, n = r.shape
    D = r - (alpha + beta * f_mean).unsqueeze(-1)
    wb = w * beta
    den = 1.0 / f_var + (wb * beta).sum()
    logdet = torch.log(w).sum() - torch.log(f_var * den)
    u = (wb.unsqueeze(-1) * D).sum(0)                    # (n,)
    quad = (w.unsqueeze(-1) * D * D).sum() - (u * u).sum() / den
    return 0.5 * (n * (K * math.log(2 * math.pi) - logdet) + quad)


def lookback_target_split(r_stocks: Tensor, r_market: Tensor, lookback_window: int, target_window: int,
                          stride: Optional[int] = None, prediction: bool = True) -> Tuple[Tensor, Tensor]:
    """Windows of (stock, market) pairs (reference `src/common.py:81-112`).

    r_stocks (K, N), r_market (N,) -> X (W, K, Tx, 2), y (W, K, Ty, 2).
    Prediction: X = the lookback, y = the following ``target_window`` days.
    Reconstruction: X = the lookback, y = its last ``target_window`` days.
    Returned tensors are views of one stacked (K, N, 2) buffer.
    """
    if stride is None:
        stride = lookback_window + target_window
    span = lookback_window + target_window if prediction else lookback_window
    K, N = r_stocks.shape
    pairs = torch.stack([r_stocks, r_market.unsqueeze(0).expand(K, N)], dim=-1)  # (K, N, 2)
    W = (N - span) // stride + 1 if N >= span else 0
    win = pairs.as_strided((W, K, span, 2), (stride * 2, N * 2, 2, 1), pairs.storage_offset())
    if prediction:
        return win[:, :, :lookback_window], win[:, :, lookback_window:]
    return win, win[:, :, lookback_window - target_window:]


def add_quadratic_features(X: Tensor, interaction_only: bool = False, include_bias: bool = False) -> Tensor:
    """[r_s, r_m, r_s·r_m] (+ [r_s², r_m²] unless ``interaction_only``) (reference `src/common.py:115-130`)."""
    rs, rm = X[..., 0], X[..., 1]
    feats = [rs, rm, rs * rm]
    if not interaction_only:
        feats += [rs * rs, rm * rm]
    if include_bias:
        feats.append(torch.ones_like(rs))
    return torch.stack(feats, dim=-1)


def ols_features(target: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """OLS targets of the future window (reference `src/common.py:132-149`).

    target (W, K, n, ≥2) -> alphas (W, K), betas (W, K), factor (W, 2) = [mean, unbiased var] of the
    market, inv_psi (W, K) = 1 / unbiased residual variance.
    """
    rs = target[..., 0]                 # (W, K, n)
    rm = target[:, 0, :, 1]             # (W, n)
    alphas, betas = ols(rm, rs)
    resid = rs - (alphas.unsqueeze(-1) + betas.unsqueeze(-1) * rm.unsqueeze(1))
    factor = torch.stack([rm.mean(-1), rm.var(-1)], dim=-1)
    inv_psi = resid.var(-1).reciprocal()
    return alphas, betas, factor, inv_psi


def append_feature(y: Tensor, feature: Tensor) -> Tensor:
    """Broadcast a per-(window, stock) value (or per-stock, shared by all windows) into a new channel of
    ``y`` (W, K, n, C) (reference `src/data.py:126-130`)."""
    W, K, n, _ = y.shape
    f = feature.reshape(-1, K)[..., None, None].expand(W, K, n, 1).to(y.dtype)
    return torch.cat([y, f], dim=-1)
