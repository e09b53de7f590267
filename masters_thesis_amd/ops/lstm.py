"""Multi-layer LSTM encoder op (reference: ``torch.nn.LSTM`` in `src/model.py:88-94,104`).

GPU path (``_LSTMStackFn``): per layer one persistent HIP recurrence kernel
(``csrc/lstm.hip``) in time-major layout with the sequence axis padded to a
multiple of 16 (``Np``) so the kernels need no per-lane bounds checks.  Layer 0's
tiny input projection (F in {3, 5}) is fused into the recurrence; deeper layers get
theirs as one time-parallel GEMM over all T*Np rows, with gate columns in the
kernels' unit-major order (``lstm_prep`` permutes W_ih / bias each step).

Backward runs the reverse-time HIP kernel (reading the fragment-ordered stash the
forward wrote, emitting unit-major dG), then ONE weight-gradient kernel per layer
(``lstm_wgrad``) that accumulates dW_ih, dW_hh and both bias gradients directly into
the parameters' ``.grad`` views (the flat gradient buffer).  The op therefore
returns ``None`` for the weights: gradient accumulation happens inside the op,
which removes the per-parameter AccumulateGrad kernels.  Padded rows carry zero
upstream gradient, hence zero dG.  Inter-layer dropout (between layers only,
train only, `src/model.py:92`) uses a saved Bernoulli mask.

CPU path: ``torch._VF.lstm`` (the exact kernel behind ``nn.LSTM``).
"""
from __future__ import annotations

from typing import List, Sequence

import torch
from torch import Tensor

from ._lib import lib, use_hip

MATMUL_PRECISION = {"highest": 0, "high": 1, "medium": 2}
FUSED_F = (3, 5)


def precision_code(p) -> int:
    if isinstance(p, int):
        return p
    if p is None:
        p = torch.get_float32_matmul_precision()
    return MATMUL_PRECISION[str(p)]


def padded_rows(n: int) -> int:
    return (n + 15) // 16 * 16


def _grad_buffer(p: Tensor) -> Tensor:
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


class _LSTMStackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, prec: int, dropout: float, training: bool, need_grad: bool, *flat: Tensor) -> Tensor:
        L = len(flat) // 4
        N, T, F = x.shape
        H = flat[1].shape[1]
        Np = padded_rows(N)
        C = lib()
        dev = x.device
        x = x.contiguous()
        saved: List[Tensor] = []
        masks: List[Tensor] = []
        prev_h = None
        for l in range(L):
            w_ih, w_hh, b_ih, b_hh = flat[4 * l: 4 * l + 4]
            hseq = torch.empty((T, Np, H), device=dev, dtype=torch.float32)
            stash = torch.empty((T * Np * 5 * H,), device=dev, dtype=torch.float32) if need_grad else None
            if l == 0 and F in FUSED_F:
                C.lstm_fwd_layer(H, prec, x, w_ih, b_ih, b_hh, None, stash, w_hh, hseq, N, Np, T)
                inp, w_um = x, w_ih
            else:
                if l == 0:
                    inp = x.new_zeros((T, Np, F))
                    inp[:, :N].copy_(x.transpose(0, 1))
                    inp = inp.view(T * Np, F)
                else:
                    inp = prev_h.view(T * Np, H)
                    if dropout > 0.0 and training:
                        mask = torch.empty_like(inp).bernoulli_(1.0 - dropout).div_(1.0 - dropout)
                        masks.append(mask)
                        inp = inp * mask
                fin = inp.shape[1]
                w_um = torch.empty((4 * H, fin), device=dev, dtype=torch.float32)
                b_um = torch.empty((4 * H,), device=dev, dtype=torch.float32)
                C.lstm_prep(w_ih, b_ih, b_hh, H, w_um, b_um)
                gx = torch.addmm(b_um, inp, w_um.t())
                C.lstm_fwd_layer(H, prec, None, None, None, None, gx, stash, w_hh, hseq, N, Np, T)
            saved += [inp, stash if stash is not None else hseq, hseq, w_um]
            prev_h = hseq
        ctx.L, ctx.H, ctx.N, ctx.Np, ctx.T, ctx.F = L, H, N, Np, T, F
        ctx.prec, ctx.dropout, ctx.training = prec, dropout, training
        ctx.params = flat  # gradients are accumulated into p.grad by the op itself
        if need_grad:
            ctx.save_for_backward(*saved, *masks)
        return prev_h[T - 1, :N]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh_last: Tensor):
        L, H, N, Np, T, F = ctx.L, ctx.H, ctx.N, ctx.Np, ctx.T, ctx.F
        C = lib()
        tensors = ctx.saved_tensors
        saved = tensors[: 4 * L]
        masks = list(tensors[4 * L:])
        dH = None
        dx = None
        dh_last = dh_last.contiguous()
        for l in range(L - 1, -1, -1):
            w_ih, w_hh, b_ih, b_hh = ctx.params[4 * l: 4 * l + 4]
            inp, stash, hseq, w_um = saved[4 * l: 4 * l + 4]
            dG = torch.empty((T, Np, 4 * H), device=dh_last.device, dtype=torch.float32)
            C.lstm_bwd_layer(H, ctx.prec, stash, w_hh, dH, None if dH is not None else dh_last, dG, N, Np, T)
            fused0 = l == 0 and F in FUSED_F
            C.lstm_wgrad(ctx.prec, dG, hseq, inp, fused0, N, Np, T, H, _grad_buffer(w_ih), _grad_buffer(w_hh),
                         _grad_buffer(b_ih), _grad_buffer(b_hh))
            dG2 = dG.view(T * Np, 4 * H)
            if l > 0:
                dinp = dG2.mm(w_um)
                if ctx.dropout > 0.0 and ctx.training:
                    dinp.mul_(masks[l - 1])
                dH = dinp.view(T, Np, H)
            elif ctx.needs_input_grad[0]:
                perm = _unit_major_rows(H, dG.device)
                dx = dG2.mm(w_ih.index_select(0, perm)).view(T, Np, F)[:, :N].transpose(0, 1)
        return (dx, None, None, None, None, *([None] * (4 * L)))


_PERM_CACHE = {}


def _unit_major_rows(H: int, device) -> Tensor:
    """perm[c'] = r for unit-major gate column c' = 4u + g and nn.LSTM row r = g*H + u."""
    key = (H, str(device))
    if key not in _PERM_CACHE:
        c = torch.arange(4 * H)
        _PERM_CACHE[key] = ((c % 4) * H + c // 4).to(device)
    return _PERM_CACHE[key]


def lstm_last_hidden(x: Tensor, weights: Sequence[Tensor], num_layers: int, dropout: float, training: bool,
                     precision=None) -> Tensor:
    """Run the stacked LSTM over batch-first ``x (N, T, F)`` and return ``h_T`` of the top layer (N, H).

    ``weights`` is nn.LSTM's flat list ``[w_ih_l0, w_hh_l0, b_ih_l0, b_hh_l0, w_ih_l1, ...]``.
    """
    if use_hip(x):
        # grad mode is off inside Function.forward: decide here whether to keep the stash
        need_grad = torch.is_grad_enabled() and any(t.requires_grad for t in (x, *weights))
        return _LSTMStackFn.apply(x, precision_code(precision), float(dropout), bool(training), need_grad, *weights)
    H = weights[1].shape[1]
    N = x.shape[0]
    h0 = x.new_zeros(num_layers, N, H)
    out, _, _ = torch._VF.lstm(x, (h0, h0), list(weights), True, num_layers, float(dropout), bool(training), False,
                               True)
    return out[:, -1, :]
