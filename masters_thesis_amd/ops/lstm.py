"""Multi-layer LSTM encoder op (reference: ``torch.nn.LSTM`` in `src/model.py:88-94,104`).

GPU path (``_LSTMStackFn``): per layer one persistent HIP recurrence kernel
(``csrc/lstm.hip``) in time-major layout; layer 0's tiny input projection (F <= 5)
is fused into the recurrence, deeper layers get their input projection as one
time-parallel GEMM over all T*N rows.  Backward runs the reverse-time HIP kernel
(which turns the stashed gates into dG in place) followed by three time-parallel
GEMMs per layer (dW_hh, dW_ih, dX) and a bias reduction.  Inter-layer dropout
(only between layers, train only, `src/model.py:92`) uses a saved Bernoulli mask.

CPU path: ``torch._VF.lstm`` (the exact kernel behind ``nn.LSTM``), so CPU runs
match the reference bit-for-bit.
"""
from __future__ import annotations

from typing import List, Sequence

import torch
from torch import Tensor

from ._lib import lib, use_hip

MATMUL_PRECISION = {"highest": 0, "high": 1, "medium": 2}


def precision_code(p) -> int:
    if isinstance(p, int):
        return p
    if p is None:
        p = torch.get_float32_matmul_precision()
    return MATMUL_PRECISION[str(p)]


class _LSTMStackFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, prec: int, dropout: float, training: bool, *flat: Tensor) -> Tensor:
        L = len(flat) // 4
        N, T, F = x.shape
        H = flat[1].shape[1]
        C = lib()
        dev = x.device
        x = x.contiguous()
        need_grad = torch.is_grad_enabled() or any(t.requires_grad for t in (x, *flat))
        saved: List[Tensor] = []
        masks: List[Tensor] = []
        inp = None
        hseq = None
        for l in range(L):
            w_ih, w_hh, b_ih, b_hh = flat[4 * l: 4 * l + 4]
            gates = torch.empty((T, N, 4 * H), device=dev, dtype=torch.float32)
            hseq = torch.empty((T, N, H), device=dev, dtype=torch.float32)
            cseq = torch.empty((T, N, H), device=dev, dtype=torch.float32)
            if l == 0 and F <= 5:
                C.lstm_fwd_layer(H, prec, x, w_ih.contiguous(), b_ih.contiguous(), b_hh.contiguous(), None, gates,
                                 w_hh.contiguous(), hseq, cseq, N, T)
                inp = x
            else:
                if l == 0:
                    inp = x.transpose(0, 1).reshape(T * N, F)
                else:
                    inp = prev_h.reshape(T * N, H)
                    if dropout > 0.0 and training:
                        mask = torch.empty_like(inp).bernoulli_(1.0 - dropout).div_(1.0 - dropout)
                        masks.append(mask)
                        inp = inp * mask
                torch.addmm(b_ih + b_hh, inp, w_ih.t(), out=gates.view(T * N, 4 * H))
                C.lstm_fwd_layer(H, prec, None, None, None, None, gates, gates, w_hh.contiguous(), hseq, cseq, N, T)
            saved += [inp, gates, hseq, cseq]
            prev_h = hseq
        ctx.L, ctx.H, ctx.N, ctx.T, ctx.F = L, H, N, T, F
        ctx.prec, ctx.dropout, ctx.training = prec, dropout, training
        ctx.n_masks = len(masks)
        if need_grad:
            ctx.save_for_backward(*flat, *saved, *masks)
        return hseq[T - 1]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh_last: Tensor):
        L, H, N, T, F = ctx.L, ctx.H, ctx.N, ctx.T, ctx.F
        C = lib()
        tensors = ctx.saved_tensors
        flat = tensors[: 4 * L]
        saved = tensors[4 * L: 8 * L]
        masks = list(tensors[8 * L:])
        grads: List[Tensor] = [None] * (4 * L)  # type: ignore[list-item]
        dH = None
        dx = None
        dh_last = dh_last.contiguous()
        for l in range(L - 1, -1, -1):
            w_ih, w_hh, _, _ = flat[4 * l: 4 * l + 4]
            inp, gates, hseq, cseq = saved[4 * l: 4 * l + 4]
            if dH is None:
                C.lstm_bwd_layer(H, ctx.prec, gates, cseq, w_hh.contiguous(), None, dh_last, N, T)
            else:
                C.lstm_bwd_layer(H, ctx.prec, gates, cseq, w_hh.contiguous(), dH, None, N, T)
            dG = gates.view(T * N, 4 * H)
            db = dG.sum(0)
            dW_hh = dG[N:].t().mm(hseq[:-1].reshape((T - 1) * N, H)) if T > 1 else torch.zeros_like(w_hh)
            if l == 0 and F <= 5:
                inp_tm = inp.transpose(0, 1).reshape(T * N, F)
            else:
                inp_tm = inp
            dW_ih = dG.t().mm(inp_tm)
            grads[4 * l: 4 * l + 4] = [dW_ih, dW_hh, db, db.clone()]
            if l > 0:
                dinp = dG.mm(w_ih)
                if ctx.dropout > 0.0 and ctx.training:
                    dinp.mul_(masks[l - 1])
                dH = dinp.view(T, N, H)
            elif ctx.needs_input_grad[0]:
                dx = dG.mm(w_ih).view(T, N, F).transpose(0, 1)
        return (dx, None, None, None, *grads)


def lstm_last_hidden(x: Tensor, weights: Sequence[Tensor], num_layers: int, dropout: float, training: bool,
                     precision=None) -> Tensor:
    """Run the stacked LSTM over batch-first ``x (N, T, F)`` and return ``h_T`` of the top layer (N, H).

    ``weights`` is nn.LSTM's flat list ``[w_ih_l0, w_hh_l0, b_ih_l0, b_hh_l0, w_ih_l1, ...]``.
    """
    if use_hip(x):
        return _LSTMStackFn.apply(x, precision_code(precision), float(dropout), bool(training), *weights)
    H = weights[1].shape[1]
    N = x.shape[0]
    h0 = x.new_zeros(num_layers, N, H)
    out, _, _ = torch._VF.lstm(x, (h0, h0), list(weights), True, num_layers, float(dropout), bool(training), False,
                               True)
    return out[:, -1, :]
