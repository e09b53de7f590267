"""Fused decoder losses (reference K5-K9: `src/model.py:45-69,176-331`, `src/common.py:50-78`).

``decoder_losses(ab, y, factor, inv_psi)`` returns ``(mse, nll, mae)`` for
``ab = [alpha | beta]`` (N, 2) and target windows ``y`` (N, n, C) with channel 0
the stock and channel 1 the market return:

* MSE decoder ``r_hat = alpha + beta * r_mkt``, mean over all N*n elements;
* Gaussian NLL with ``mu = alpha + beta * f_mean`` and the Woodbury inverse
  covariance, evaluated in closed form:

      w = diag(Psi^-1), s = sum w b^2, den = 1/f_var + s
      logdet Sigma^-1 = sum ln w - ln(f_var * den)
      u_t = sum_i w_i b_i D_it,  quad = sum w D^2 - sum_t u_t^2 / den
      NLL = 0.5 * (n (K ln 2pi - logdet) + quad)

  with analytic gradients (U1 = sum u_t, U2 = sum u_t^2, SD_i = sum_t D_it,
  UD_i = sum_t u_t D_it):

      dNLL/da_i = -w_i SD_i + w_i b_i U1 / den
      dNLL/db_i = n w_i b_i / den - f_mean (w_i SD_i - w_i b_i U1 / den)
                  - w_i UD_i / den + U2 w_i b_i / den^2

* MAE (test metric, `src/model.py:139`), no gradient.

Batch semantics: ``nll_mode='reference'`` reproduces the reference exactly (one
Gaussian over all B*K sequences using window 0's factor);
``'per_window'`` sums the per-window NLLs (the statistically correct batched loss).
The GPU path is one HIP kernel (``csrc/losses.hip``) that also emits the
gradients, so backward is a single tiny elementwise kernel.
"""
from __future__ import annotations

import math
from typing import Tuple

import torch
from torch import Tensor

from ._lib import lib, use_hip

LOG2PI = math.log(2 * math.pi)


def _windows(N: int, K: int, B: int, nll_mode: str) -> Tuple[int, int, int]:
    if nll_mode == "per_window":
        return B, K, 2
    return 1, N, 0


class _DecoderLossesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ab: Tensor, y: Tensor, factor: Tensor, inv_psi: Tensor, windows: int, kwin: int,
                factor_stride: int, want_nll: bool):
        C = lib()
        N = ab.shape[0]
        out = torch.empty(4, device=ab.device, dtype=torch.float32)
        g = torch.empty((2, N, 2), device=ab.device, dtype=torch.float32)
        C.decoder_losses(ab.contiguous(), y, factor, inv_psi, windows, kwin, factor_stride, bool(want_nll), out, g[0],
                         g[1])
        ctx.save_for_backward(g)
        ctx.want_nll = bool(want_nll)
        mse, nll, mae = out[0], out[1], out[2]
        ctx.mark_non_differentiable(mae)
        return mse, nll, mae

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_mse: Tensor, g_nll: Tensor, g_mae: Tensor):
        (g,) = ctx.saved_tensors
        gout = torch.stack([
            g_mse if g_mse is not None else g.new_zeros(()),
            g_nll if g_nll is not None else g.new_zeros(()),
        ]).contiguous()
        dab = torch.empty_like(g[0])
        lib().decoder_losses_bwd(gout, g[0], g[1], dab, ctx.want_nll and g_nll is not None)
        return dab, None, None, None, None, None, None, None


def woodbury_nll_torch(alpha: Tensor, beta: Tensor, f_mean: Tensor, f_var: Tensor, inv_psi: Tensor,
                       r: Tensor) -> Tensor:
    """Closed-form NLL in PyTorch ops (CPU path; autograd supplies the gradients)."""
    w, b = inv_psi, beta
    K, n = r.shape
    D = r - (alpha + b * f_mean).unsqueeze(-1)
    den = 1.0 / f_var + (w * b * b).sum()
    logdet = torch.log(w).sum() - torch.log(f_var * den)
    u = ((w * b).unsqueeze(-1) * D).sum(0)
    quad = (w.unsqueeze(-1) * D * D).sum() - (u * u).sum() / den
    return 0.5 * (n * (K * LOG2PI - logdet) + quad)


def decoder_losses(ab: Tensor, y: Tensor, factor: Tensor, inv_psi: Tensor, *, batch_windows: int = 1,
                   want_nll: bool = True, nll_mode: str = "reference") -> Tuple[Tensor, Tensor, Tensor]:
    """(mse, nll, mae) for ``ab (N,2)``, ``y (N, n, C)``, ``factor (B, 2)``, ``inv_psi (N,)``.

    ``batch_windows`` = B, the number of windows flattened into N (N = B*K).
    """
    N = ab.shape[0]
    K = N // batch_windows
    windows, kwin, fstride = _windows(N, K, batch_windows, nll_mode)
    if use_hip(ab):
        return _DecoderLossesFn.apply(ab, y.contiguous(), factor.contiguous(), inv_psi.contiguous(), windows, kwin,
                                      fstride, want_nll)
    alpha, beta = ab[:, 0], ab[:, 1]
    r, rm = y[..., 0], y[..., 1]
    e = alpha.unsqueeze(-1) + beta.unsqueeze(-1) * rm - r
    mse = (e * e).mean()
    mae = e.detach().abs().mean()
    if not want_nll:
        return mse, torch.zeros((), dtype=mse.dtype, device=mse.device), mae
    fac = factor.reshape(-1)
    nll = 0.0
    for wdw in range(windows):
        sl = slice(wdw * kwin, (wdw + 1) * kwin)
        fm, fv = fac[wdw * fstride], fac[wdw * fstride + 1]
        nll = nll + woodbury_nll_torch(alpha[sl], beta[sl], fm, fv, inv_psi.reshape(-1)[sl], r[sl])
    return mse, nll, mae
