"""Fused alpha/beta heads + decoder losses (reference K4-K9: `src/model.py:45-69,96-108,176-331`,
`src/common.py:50-78`).

``heads_losses(h, wa, ba, wb, bb, y, factor, inv_psi)`` evaluates the two
``Linear(H, 1)`` heads on the encoder state ``h`` (N, H) and returns
``(ab, mse, nll, mae, total)`` for target windows ``y`` (N, n, C) (channel 0 the
stock, channel 1 the market return):

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

* MAE (test metric, `src/model.py:139`), no gradient;
* ``total = c_nll * NLL + c_mse * MSE`` (the model's training loss).

Batch semantics: ``nll_mode='reference'`` reproduces the reference exactly (one
Gaussian over all B*K sequences using window 0's factor);
``'per_window'`` sums the per-window NLLs (the statistically correct batched loss).

GPU path: ONE HIP kernel (``csrc/losses.hip``) computes the heads, every loss, the
per-sequence gradients and adds the epoch metric sums into ``acc`` (8 float64:
sse, count, nll_sum, nll_updates, total_sum, total_weight, sae, count); backward is
one kernel producing dh and accumulating the head weight gradients directly into
the parameters' ``.grad`` views.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
from torch import Tensor

from ._lib import lib, use_hip


def set_deterministic(flag: bool) -> None:
    """Deterministic mode: the wide-head backward (N * H > 32768: extras encoders, large batches) sums its per-block
    head-parameter partials in block order (csrc/losses.hip heads_part_reduce_kernel) instead of f32 atomics."""
    try:
        lib().set_heads_deterministic(bool(flag))
    except Exception:  # CPU-only process: the PyTorch path is deterministic already
        pass

LOG2PI = math.log(2 * math.pi)


def _windows(N: int, B: int, nll_mode: str) -> Tuple[int, int, int]:
    if nll_mode == "per_window":
        return B, N // B, 2
    return 1, N, 0


def _c(t: Optional[Tensor]) -> Optional[Tensor]:
    return None if t is None else t.contiguous().float()


def _grad_buffer(p: Tensor) -> Tensor:
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


class _HeadsLossesFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h: Tensor, wa: Tensor, ba: Tensor, wb: Tensor, bb: Tensor, y: Tensor, factor: Tensor,
                inv_psi: Tensor, windows: int, kwin: int, fstride: int, want_nll: bool, c_nll: float, c_mse: float,
                batch_weight: float, acc: Optional[Tensor]):
        C = lib()
        N = h.shape[0]
        dev = h.device
        out = torch.empty(4, device=dev, dtype=torch.float32)
        g = torch.empty((2, N, 2), device=dev, dtype=torch.float32)
        ab = torch.empty((N, 2), device=dev, dtype=torch.float32)
        C.heads_losses(h, wa, ba, wb, bb, ab, y, factor, inv_psi, windows, kwin, fstride, bool(want_nll),
                       float(c_nll), float(c_mse), float(batch_weight), out, g[0], g[1], acc)
        ctx.save_for_backward(g, h)
        ctx.params = (wa, ba, wb, bb)
        ctx.want_nll, ctx.c_nll, ctx.c_mse = bool(want_nll), float(c_nll), float(c_mse)
        mse, nll, mae, total = out[0], out[1], out[2], out[3]
        ctx.mark_non_differentiable(ab, mae)
        ctx.set_materialize_grads(False)
        return ab, mse, nll, mae, total

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_ab, g_mse, g_nll, g_mae, g_total):
        g, h = ctx.saved_tensors
        wa, ba, wb, bb = ctx.params
        dh = torch.empty_like(h) if ctx.needs_input_grad[0] else None
        lib().heads_losses_bwd(_c(g_mse), _c(g_nll), _c(g_total), ctx.c_nll, ctx.c_mse, g[0], g[1], ctx.want_nll, h, wa, wb, dh, None,
                               _grad_buffer(wa), _grad_buffer(ba), _grad_buffer(wb), _grad_buffer(bb))
        return (dh,) + (None,) * 15


class _DecoderLossesFn(torch.autograd.Function):
    """Losses from a precomputed ``ab`` (N, 2) — for encoders whose heads are not fused."""

    @staticmethod
    def forward(ctx, ab: Tensor, y: Tensor, factor: Tensor, inv_psi: Tensor, windows: int, kwin: int, fstride: int,
                want_nll: bool, c_nll: float, c_mse: float, batch_weight: float, acc: Optional[Tensor]):
        C = lib()
        N = ab.shape[0]
        out = torch.empty(4, device=ab.device, dtype=torch.float32)
        g = torch.empty((2, N, 2), device=ab.device, dtype=torch.float32)
        C.decoder_losses(ab.contiguous(), y, factor, inv_psi, windows, kwin, fstride, bool(want_nll), float(c_nll),
                         float(c_mse), float(batch_weight), out, g[0], g[1], acc)
        ctx.save_for_backward(g)
        ctx.want_nll, ctx.c_nll, ctx.c_mse = bool(want_nll), float(c_nll), float(c_mse)
        mse, nll, mae, total = out[0], out[1], out[2], out[3]
        ctx.mark_non_differentiable(mae)
        ctx.set_materialize_grads(False)
        return mse, nll, mae, total

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_mse, g_nll, g_mae, g_total):
        (g,) = ctx.saved_tensors
        dab = torch.empty_like(g[0])
        lib().heads_losses_bwd(_c(g_mse), _c(g_nll), _c(g_total), ctx.c_nll, ctx.c_mse, g[0], g[1], ctx.want_nll, None, None, None, None, dab,
                               None, None, None, None)
        return (dab,) + (None,) * 11


# --------------------------------------------------------------------------- CPU (PyTorch) path
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


def _losses_torch(ab, y, factor, inv_psi, windows, kwin, fstride, want_nll, c_nll, c_mse, batch_weight, acc):
    alpha, beta = ab[:, 0], ab[:, 1]
    r, rm = y[..., 0], y[..., 1]
    e = alpha.unsqueeze(-1) + beta.unsqueeze(-1) * rm - r
    mse = (e * e).mean()
    mae = e.detach().abs().mean()
    nll = torch.zeros((), dtype=mse.dtype, device=mse.device)
    if want_nll:
        fac = factor.reshape(-1)
        ip = inv_psi.reshape(-1)
        for wdw in range(windows):
            sl = slice(wdw * kwin, (wdw + 1) * kwin)
            nll = nll + woodbury_nll_torch(alpha[sl], beta[sl], fac[wdw * fstride], fac[wdw * fstride + 1], ip[sl],
                                           r[sl])
    total = c_nll * nll + c_mse * mse
    if acc is not None:
        with torch.no_grad():
            cnt = float(e.numel())
            acc += torch.tensor([float((e * e).sum()), cnt, float(nll), 1.0, float(total) * batch_weight,
                                 batch_weight, float(e.abs().sum()), cnt], dtype=acc.dtype, device=acc.device)
    return mse, nll, mae, total


# --------------------------------------------------------------------------- public API
def heads_losses(h: Tensor, wa: Tensor, ba: Tensor, wb: Tensor, bb: Tensor, y: Tensor, factor: Tensor,
                 inv_psi: Tensor, *, batch_windows: int = 1, want_nll: bool = True, nll_mode: str = "reference",
                 c_nll: float = 0.0, c_mse: float = 1.0, acc: Optional[Tensor] = None):
    """Returns ``(ab, mse, nll, mae, total)``; ``wa``/``wb`` are the (1, H) head weights, ``ba``/``bb`` (1,)."""
    N = h.shape[0]
    windows, kwin, fstride = _windows(N, batch_windows, nll_mode)
    if use_hip(h):
        return _HeadsLossesFn.apply(h.contiguous(), wa, ba, wb, bb, y.contiguous(), factor.contiguous(),
                                    inv_psi.contiguous(), windows, kwin, fstride, want_nll, c_nll, c_mse,
                                    float(batch_windows), acc)
    ab = torch.addmm(torch.cat([ba, bb]), h, torch.cat([wa, wb], 0).t())
    mse, nll, mae, total = _losses_torch(ab, y, factor, inv_psi, windows, kwin, fstride, want_nll, c_nll, c_mse,
                                         float(batch_windows), acc)
    return ab, mse, nll, mae, total


def decoder_losses(ab: Tensor, y: Tensor, factor: Tensor, inv_psi: Tensor, *, batch_windows: int = 1,
                   want_nll: bool = True, nll_mode: str = "reference", c_nll: float = 0.0, c_mse: float = 1.0,
                   acc: Optional[Tensor] = None, with_total: bool = False):
    """(mse, nll, mae[, total]) for ``ab (N,2)``, ``y (N, n, C)``, ``factor (B, 2)``, ``inv_psi (N,)``."""
    N = ab.shape[0]
    windows, kwin, fstride = _windows(N, batch_windows, nll_mode)
    if use_hip(ab):
        res = _DecoderLossesFn.apply(ab, y.contiguous(), factor.contiguous(), inv_psi.contiguous(), windows, kwin,
                                     fstride, want_nll, c_nll, c_mse, float(batch_windows), acc)
    else:
        res = _losses_torch(ab, y, factor, inv_psi, windows, kwin, fstride, want_nll, c_nll, c_mse,
                            float(batch_windows), acc)
    return res if with_total else res[:3]


# Above this many sequences the one-workgroup training decoder loses to the grid decoder path (heads / losses /
# head-backward kernels over the whole chip): at N = 800 (B = 8 windows) heads_losses_train_kernel took 185 us per
# step; with the grid path the LSTM small B = 8 step went 0.349 -> 0.334 ms, the combined-loss one 0.421 -> 0.403,
# transformer B = 8 2.186 -> 2.133 (profiles/r5_decoder_maxn_ab.txt, cap 256: B <= 2 windows keep the one-launch
# decoder and with it the LSTM's 4-launch fused step; the register-resident decoder covers N <= 128).
TRAIN_DECODER_MAX_N = 256


def train_decoder_fits(N: int, n: int, H: int = 0) -> bool:
    """Whether :func:`heads_losses_train`'s one-workgroup kernel takes (N sequences, n target days) -- and is the
    faster choice (N <= :data:`TRAIN_DECODER_MAX_N`)."""
    if N > TRAIN_DECODER_MAX_N:
        return False
    ut = ((n + 3) & ~3) + 16 * n  # u_t + one partial row per wave (csrc/losses.hip ut_floats)
    base = (3 * 2 * ((N + 1) & ~1) + ((ut + 3) & ~3)) * 4
    return base + N * n * 8 + N * H * 4 <= 96 * 1024 or base <= 60 * 1024


def heads_losses_train(h: Tensor, wa: Tensor, ba: Tensor, wb: Tensor, bb: Tensor, y: Tensor, factor: Tensor,
                       inv_psi: Tensor, *, batch_windows: int = 1, want_nll: bool = True, nll_mode: str = "reference",
                       c_nll: float = 0.0, c_mse: float = 1.0, acc: Optional[Tensor] = None,
                       grads: Tuple[Tensor, Tensor, Tensor, Tensor], out: Optional[Tensor] = None,
                       dh: Optional[Tensor] = None):
    """The training step's decoder without autograd, ONE HIP launch (``csrc/losses.hip``
    ``heads_losses_train_kernel``): heads, losses + metrics into ``acc``, the encoder gradient ``dh`` = d total /
    d h (the loss is the step's root: upstream gradient 1) and the head gradients accumulated into ``grads`` =
    (g_wa, g_ba, g_wb, g_bb).  Returns ``(out, dh)`` with ``out = [mse, nll, mae, total]``, or None when the
    problem is too large for the one-workgroup kernel (use :func:`heads_losses` + autograd then)."""
    N, H = h.shape
    windows, kwin, fstride = _windows(N, batch_windows, nll_mode)
    if out is None:
        out = torch.empty(4, device=h.device, dtype=torch.float32)
    if dh is None:
        dh = torch.empty((N, H), device=h.device, dtype=torch.float32)
    ok = lib().heads_losses_train(h.contiguous(), wa, ba, wb, bb, y.contiguous(), factor.contiguous(),
                                  inv_psi.contiguous(), windows, kwin, fstride, bool(want_nll), float(c_nll),
                                  float(c_mse), float(batch_windows), out, acc, dh, *grads)
    return (out, dh) if ok else None
