"""MLP and transformer encoder ops for the ``BASELINE.json`` north-star extras (bf16-mixed on MI355X; fp32 under
``32-true``).

Not in the reference (it only has the LSTM, `src/model.py:88-94`); the north star asks for the
``src/model.py`` forward path as Linear/GEMM+bias, GELU and LayerNorm/RMSNorm HIP kernels and a
transformer-encoder config with attention + RMSNorm + RoPE kernels.

GPU path = one autograd Function per encoder, built from four hand-written HIP kernels:

* ``gemm_bf16`` (``csrc/gemm.hip``) -- MFMA GEMM whose three layouts cover forward ``X W^T``,
  input gradient ``dY W`` and weight gradient ``dY^T X`` with no transposed copies; epilogues fuse
  bias, GELU (saving its input), dropout, GELU', the fp32 residual add, the fp32 weight-gradient
  accumulation straight into the flat gradient buffer and the bias gradient;
* ``norm`` (``csrc/norm.hip``) -- LayerNorm / RMSNorm forward and backward (dropout, GELU' and the
  residual-stream gradient fused into the backward, dgamma/dbeta accumulated);
* ``attention`` (``csrc/attention.hip``) -- RoPE attention, one wave per (sequence, head);
* ``cast_pad`` -- fp32 master weights -> zero-padded bf16 operands, once per step.

Precision: fp32 master weights (FlatParameters) and fp32 residual stream / gradients, bf16 GEMM
operands with fp32 accumulation ("bf16-mixed", matmul precision "medium").  Under ``32-true`` (matmul precision
"high" / "highest") both encoders run fp32 HIP paths instead (``_MlpEncoderF32Fn`` / ``_TransformerEncoderF32Fn``:
``gemm_f32x`` bf16x3 / exact-f32 MFMA GEMMs, fp32 norms, fp32 attention ``csrc/attention_f32.hip``), so the
trainer's precision is never silently lowered.  Like the LSTM op, the weights' gradients are accumulated inside the
op and ``None`` is returned for them.

CPU path: the same architectures in plain fp32 PyTorch (``mlp_reference`` / ``transformer_reference``),
which also serve as the numerics oracle of the GPU tests.
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Sequence

import torch
import torch.nn.functional as Fn
from torch import Tensor

from ..parallel.overlap import grad_ready
from .optim import register_grad_producer
from ._lib import lib, use_hip

EPI_BIAS, EPI_GELU, EPI_RESID, EPI_ACCUM, EPI_DROPOUT, EPI_DGELU = 1, 2, 4, 8, 16, 32
ROPE_BASE = 10000.0
LN_EPS = 1e-5
RMS_EPS = 1e-6


def _r8(n: int) -> int:
    return (n + 7) // 8 * 8


def _r16(n: int) -> int:
    return (n + 15) // 16 * 16


# --------------------------------------------------------------------------------------------------
# thin launchers
# --------------------------------------------------------------------------------------------------
def gemm(mode: int, A: Tensor, B: Tensor, M: int, N: int, K: int, lda: int, ldb: int, *, flags: int = 0,
         alpha: float = 1.0, bias=None, resid=None, aux_in=None, seed=None, drop_p: float = 0.0, out_bf16=None,
         out_f32=None, aux_pre=None, ldc: Optional[int] = None, n_store: int = 0, ksplit: int = 1,
         bias_grad=None, defer: bool = False, group: bool = False) -> None:
    """``defer`` (weight-gradient GEMMs): hold the launch back and run it together with the NEXT gemm call (its
    input-gradient partner, which reads the same dY) as one paired launch (csrc/gemm.hip); ``gemm_flush()``
    launches a held-back GEMM alone.  ``group`` (weight-gradient GEMMs): queue it for one grouped launch of every
    queued weight gradient at ``gemm_group_flush()`` (``ksplit`` 1: no split-K, else the flush picks it)."""
    lib().gemm_bf16(mode, A, B, M, N, K, lda, ldb, alpha, flags, bias, resid, aux_in, seed, drop_p, out_bf16,
                    out_f32, aux_pre, N if ldc is None else ldc, n_store, ksplit, bias_grad,
                    2 if group else int(bool(defer)))


def gemm_flush() -> None:
    lib().gemm_flush()


def gemm_group_flush() -> None:
    lib().gemm_group_flush()


_DETERMINISTIC = [False]


def set_deterministic(flag: bool) -> None:
    """Deterministic mode: weight-gradient GEMMs without split-K (no cross-workgroup f32 atomics).  The
    LayerNorm/RMSNorm parameter gradients still reduce across workgroups with atomics (csrc/norm.hip)."""
    _DETERMINISTIC[0] = bool(flag)


# workgroup target of a split-K weight gradient: 128, so that a (weight-gradient,
# input-gradient) pair of the transformer (~128 + ~196 workgroups) runs as one wave of workgroups and the fp32 atomics
# halve -- transformer B=1 0.565 -> 0.528 ms; 64: 0.586, 256: 0.565, 512: 0.638 (profiles/r4_wgrad_wgs_sweep.txt)
_WGRAD_WGS = 128


def wgrad_split(M: int, N: int, K: int) -> int:
    """Split-K count for a weight-gradient GEMM: ~_WGRAD_WGS workgroups, >= 4 k-slices of 32 each."""
    if _DETERMINISTIC[0]:
        return 1
    tiles = -(-M // 64) * -(-N // 64)
    return max(1, min(_WGRAD_WGS // max(tiles, 1), K // 128))


def cast_pad(srcs: Sequence[Tensor], dsts: Sequence[Tensor], seeds: Optional[Tensor] = None) -> None:
    """fp32 -> zero-padded bf16 operands (rows and columns past the source are zeros); ``seeds``: the encoder's
    dropout seeds, advanced by the same launch (one fresh counter-hash seed per site and step, no ATen kernel)."""
    C = lib()
    for i in range(0, len(srcs), 16):
        C.cast_pad(list(srcs[i:i + 16]), list(dsts[i:i + 16]), seeds if i == 0 else None)


def _padded_bf16(w: Tensor, cols_p: int) -> Tensor:
    return torch.empty((w.shape[0], cols_p), device=w.device, dtype=torch.bfloat16)


def _row_dtype(D: int) -> torch.dtype:
    """Storage of a GEMM -> norm row tensor (activation or its gradient): fp32.  bf16 rows measured no faster --
    r3: mlp_large B=64 1.277 -> 1.327 ms (profiles/r3_bf16_rows_negative.txt); r5, with the bf16-row form of the wide
    norm backward: 1.1318 -> 1.1293 ms, within noise, at a bf16 rounding of every LayerNorm input
    (profiles/r5_bf16_rows_negative.txt)."""
    return torch.float32


def _gelu_in_norm(D: int) -> bool:
    """bf16 MLP layer of width D: the GEMM stores only the bf16 pre-activation and the wide norm kernels apply the
    GELU on load (csrc/norm.hip NormArgs::gelu_x) -- the LayerNorm input is gelu(bf16 pre-activation), as under
    autocast, instead of an fp32 GELU output written by the GEMM and read back by both norm kernels (78 -> 26 MB
    written per mlp_large layer).  The wide kernels' widths: D = 1024 / 2048."""
    return D in (1024, 2048)


def _row_out(t: Tensor) -> dict:
    return {"out_bf16": t} if t.dtype == torch.bfloat16 else {"out_f32": t}


def _grad_view(p: Tensor) -> Tensor:
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


# --------------------------------------------------------------------------------------------------
# MLP encoder:  z_0 = flatten(x);  z_{i+1} = dropout_i(Norm_i(GELU(z_i W_i^T + b_i)))   (no dropout last)
# --------------------------------------------------------------------------------------------------
def mlp_reference(x: Tensor, params: Sequence[Tensor], num_layers: int, norm: str, dropout: float,
                  training: bool) -> Tensor:
    z = x.flatten(1)
    per = 4 if norm == "layernorm" else 3
    for i in range(num_layers):
        w, b = params[per * i], params[per * i + 1]
        z = Fn.gelu(Fn.linear(z, w, b))
        if norm == "layernorm":
            z = Fn.layer_norm(z, (z.shape[-1],), params[per * i + 2], params[per * i + 3], LN_EPS)
        else:
            z = Fn.rms_norm(z, (z.shape[-1],), params[per * i + 2], RMS_EPS)
        if i < num_layers - 1 and dropout > 0 and training:
            z = Fn.dropout(z, dropout, True)
    return z


class _MlpEncoderFn(torch.autograd.Function):
    """bf16 MLP encoder.  ``n_heads`` = 4: the last four of ``params`` are the alpha / beta heads (wa, ba, wb, bb)
    and they are FUSED into the last layer's norm kernels (csrc/norm.hip NormArgs::ab): the forward returns
    ab = [h wa^T + ba | h wb^T + bb] (N, 2) without writing h, the backward takes d(ab) and forms the last layer's dy =
    d_alpha wa + d_beta wb on the fly, accumulating the head-weight gradients from h recomputed as xhat gamma + beta
    -- the heads kernel, the head backward kernel, and h / dh written and read back (52 MB each for mlp_large) go."""

    @staticmethod
    def forward(ctx, x, seeds, num_layers, norm, dropout, training, need_grad, n_heads, *params):
        heads = params[len(params) - n_heads:] if n_heads else None
        params = params[:len(params) - n_heads]
        dev = x.device
        N = x.shape[0]
        Mp = _r16(N)
        L = num_layers
        per = 4 if norm == "layernorm" else 3
        rms = norm != "layernorm"
        drop = dropout > 0 and training
        K0 = x[0].numel()
        dims = [K0] + [params[per * i].shape[0] for i in range(L)]
        # K padded to 32: the first layer's K = 60 x 3 = 180 -> 192 runs on the 256 x 256 kernel (32-deep k-tiles)
        # instead of the 128-tile path (6400 x 2048 x 184: 43 us at 174 TFLOP/s, r3 trace)
        kp = [-(-d // 32) * 32 for d in dims]
        X0 = torch.empty((Mp, kp[0]), device=dev, dtype=torch.bfloat16)
        wb = [_padded_bf16(params[per * i], kp[i]) for i in range(L)]
        cast_pad([x.reshape(N, K0)] + [params[per * i] for i in range(L)], [X0] + wb, seeds if drop else None)
        Xs, pres, acts, means, rstds = [X0], [], [], [], []
        h = None
        for i in range(L):
            D = dims[i + 1]
            assert D % 8 == 0, "MLP hidden size must be a multiple of 8"
            pre = torch.empty((Mp, D), device=dev, dtype=torch.bfloat16)
            if _gelu_in_norm(D):
                # the GEMM stores only the bf16 pre-activation; both norm kernels apply the GELU on load
                act = None
                gemm(0, Xs[i], wb[i], Mp, D, kp[i], kp[i], kp[i], flags=EPI_BIAS, bias=params[per * i + 1],
                     out_bf16=pre)
            else:
                # the GELU output rows are fp32 (_row_dtype)
                act = torch.empty((Mp, D), device=dev, dtype=_row_dtype(D))
                gemm(0, Xs[i], wb[i], Mp, D, kp[i], kp[i], kp[i], flags=EPI_BIAS | EPI_GELU,
                     bias=params[per * i + 1], aux_pre=pre, **_row_out(act))
            mean = None if rms else torch.empty(Mp, device=dev, dtype=torch.float32)
            rstd = torch.empty(Mp, device=dev, dtype=torch.float32)
            last = i == L - 1
            y = torch.empty((Mp, D), device=dev, dtype=torch.bfloat16) if not last else None
            hk = {}
            if last and heads is not None:
                assert act is None, "fused heads need the GELU-on-load norm (ops.extras._gelu_in_norm)"
                h = None
                ab = torch.empty((Mp, 2), device=dev, dtype=torch.float32)
                hk = dict(hw_a=heads[0], hb_a=heads[1], hw_b=heads[2], hb_b=heads[3], ab=ab)
            elif last:
                h = torch.empty((Mp, D), device=dev, dtype=torch.float32)
            lib().norm(False, pre if act is None else act, D, Mp, D, rms, RMS_EPS if rms else LN_EPS,
                       params[per * i + 2], None if rms else params[per * i + 3], y, h if last else None, mean, rstd,
                       seeds[i:i + 1] if (drop and not last) else None, float(dropout), None, None, None, None, None,
                       None, None, gelu_x=act is None, **hk)
            pres.append(pre)
            acts.append(act)
            means.append(mean)
            rstds.append(rstd)
            if not last:
                Xs.append(y)
        ctx.meta = (N, Mp, L, per, rms, drop, float(dropout), dims, kp)
        ctx.params = params
        ctx.heads = heads
        ctx.wb = wb
        ctx.seeds = seeds
        if need_grad:
            ctx.save_for_backward(*Xs, *pres, *acts)
            ctx.stats = (means, rstds)
        return ab[:N] if heads is not None else h[:N]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh):
        N, Mp, L, per, rms, drop, p, dims, kp = ctx.meta
        params, wb = ctx.params, ctx.wb
        saved = ctx.saved_tensors
        Xs, pres, acts = saved[:L], saved[L:2 * L], saved[2 * L:]
        means, rstds = ctx.stats
        dev = dh.device
        heads = ctx.heads
        base = dh._base
        if heads is not None:
            dab = dh.contiguous().float()  # d(alpha, beta): the last layer's dy is formed in its norm kernel
            dy = None
        elif Mp == N and dh.dtype == torch.float32 and dh.is_contiguous():
            dy = dh  # read-only below: no zero-fill + copy of the output gradient
        elif (getattr(base, "_mta_zero_pad", False) and base.shape == (Mp, dims[-1]) and base.is_contiguous()
              and dh.data_ptr() == base.data_ptr() and dh.shape[0] == N):
            dy = base  # the fused step's decoder wrote dh into a padded buffer with zero pad rows
        else:
            dy = torch.empty((Mp, dims[-1]), device=dev, dtype=torch.float32)
            dy[:N].copy_(dh)
            dy[N:].zero_()
        for i in range(L - 1, -1, -1):
            D, Din = dims[i + 1], dims[i]
            dpre = torch.empty((Mp, D), device=dev, dtype=torch.bfloat16)
            dropped = drop and i < L - 1
            hk = {}
            if heads is not None and i == L - 1:
                wa, ba, wb_, bb = heads
                hk = dict(hw_a=wa, hb_a=ba, hw_b=wb_, hb_b=bb, ab=dab, ab_rows=N, g_wa=_grad_view(wa),
                          g_wb=_grad_view(wb_))
            if acts[i] is None:
                lib().norm_defer()  # dgamma / dbeta (+ head) partials: one reduction launch for all layers at the end
            lib().norm(True, pres[i] if acts[i] is None else acts[i], D, Mp, D, rms, RMS_EPS if rms else LN_EPS,
                       params[per * i + 2], None if rms else params[per * i + 3], None, None, means[i], rstds[i],
                       ctx.seeds[i:i + 1] if dropped else None, p, dy, None, pres[i], dpre, None,
                       _grad_view(params[per * i + 2]), None if rms else _grad_view(params[per * i + 3]),
                       gelu_x=acts[i] is None, **hk)
            if hk:  # head biases: ordered column sums of d(alpha, beta) (the head weights' sums: at norm_flush)
                lib().pair_colsum(dab, N, _grad_view(ba), _grad_view(bb))
            # dW_i += dPre^T X_i (fp32 straight into the flat gradient buffer), db_i += colsum(dPre).  A big dW_i is
            # a gradient PRODUCER of the fused optimizer (ops/optim.py register_grad_producer): its split-K reduce
            # overwrites the range and leaves the clip-norm partials, so the update neither zeroes nor re-reads it
            parts = register_grad_producer(_grad_view(params[per * i])) if D * Din >= (1 << 20) else None
            if parts is not None:
                lib().gemm_grad_producer(parts, True)
            gemm(2, dpre, Xs[i], D, kp[i], Mp, D, kp[i], flags=EPI_ACCUM, out_f32=_grad_view(params[per * i]),
                 ldc=Din, n_store=Din, ksplit=wgrad_split(D, kp[i], Mp), bias_grad=_grad_view(params[per * i + 1]),
                 defer=i > 0 and parts is None)  # paired with the input-gradient GEMM below (same dPre)
            if i > 0:
                dy = torch.empty((Mp, Din), device=dev, dtype=_row_dtype(Din))
                gemm(1, dpre, wb[i], Mp, Din, D, D, kp[i], **_row_out(dy))
            # W_i, b_i final (their GEMM is launched: deferred ones go with the input-gradient GEMM above)
            grad_ready(params[per * i].grad, params[per * i + 1].grad)
        gemm_flush()
        lib().norm_flush()  # the deferred norm-parameter (and head-weight) reductions of every layer: one launch
        norm_grads = [t.grad for i in range(L) for t in params[per * i + 2:per * i + per]]
        grad_ready(*norm_grads, *([t.grad for t in heads] if heads is not None else []))
        return (None,) * (8 + len(params) + (4 if heads is not None else 0))


# --------------------------------------------------------------------------------------------------
# 32-true MLP encoder on HIP kernels: fp32 activations and gradients, every GEMM on csrc/gemm_f32.hip
# (mta_gemm_f32x) at the matmul precision the trainer resolved -- "high": bf16x3 (hi*hi + hi*lo + lo*hi,
# ~fp32-accurate), "highest": the exact-f32 MFMA -- LayerNorm / RMSNorm + dropout on csrc/norm.hip in fp32, the
# GELU' of the backward fused into the norm backward (fp32 GELU input), bias gradients by an ordered column sum.
# Reference math: mlp_reference (the same architecture in fp32 PyTorch).
# --------------------------------------------------------------------------------------------------
F32X_BIAS, F32X_GELU, F32X_DGELU, F32X_ACCUM, F32X_RESID, F32X_DROPOUT = 1, 2, 4, 8, 16, 32
_F32_PREC = {"highest": 0, "high": 1, "bf16x3": 1}


class _MlpEncoderF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, seeds, num_layers, norm, dropout, training, need_grad, prec, *params):
        dev = x.device
        N = x.shape[0]
        L = num_layers
        per = 4 if norm == "layernorm" else 3
        rms = norm != "layernorm"
        drop = dropout > 0 and training
        C = lib()
        if drop:
            C.seeds_advance(seeds)  # one fresh counter-hash mask per site and step (the bf16 path: in cast_pad)
        z = x.reshape(N, -1)
        Xs, pres, acts, means, rstds = [z], [], [], [], []
        for i in range(L):
            w, b = params[per * i], params[per * i + 1]
            D, K = w.shape
            pre = torch.empty((N, D), device=dev, dtype=torch.float32)
            act = torch.empty((N, D), device=dev, dtype=torch.float32)
            C.gemm_f32x(prec, z, False, K, w, False, K, act, D, D, N, D, K, F32X_BIAS | F32X_GELU, b, pre)
            mean = None if rms else torch.empty(N, device=dev, dtype=torch.float32)
            rstd = torch.empty(N, device=dev, dtype=torch.float32)
            y = torch.empty((N, D), device=dev, dtype=torch.float32)
            C.norm(False, act, D, N, D, rms, RMS_EPS if rms else LN_EPS, params[per * i + 2],
                   None if rms else params[per * i + 3], None, y, mean, rstd,
                   seeds[i:i + 1] if (drop and i < L - 1) else None, float(dropout), None, None, None, None, None,
                   None, None)
            pres.append(pre)
            acts.append(act)
            means.append(mean)
            rstds.append(rstd)
            z = y
            if i < L - 1:
                Xs.append(y)
        ctx.meta = (N, L, per, rms, drop, float(dropout), prec)
        ctx.params = params
        ctx.seeds = seeds
        if need_grad:
            ctx.save_for_backward(*Xs, *pres, *acts)
            ctx.stats = (means, rstds)
        return z

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh):
        N, L, per, rms, drop, p, prec = ctx.meta
        params = ctx.params
        saved = ctx.saved_tensors
        Xs, pres, acts = saved[:L], saved[L:2 * L], saved[2 * L:]
        means, rstds = ctx.stats
        C = lib()
        dy = dh.contiguous().float()
        for i in range(L - 1, -1, -1):
            w, b = params[per * i], params[per * i + 1]
            D, K = w.shape
            dpre = torch.empty((N, D), device=dh.device, dtype=torch.float32)
            dropped = drop and i < L - 1
            C.norm(True, acts[i], D, N, D, rms, RMS_EPS if rms else LN_EPS, params[per * i + 2],
                   None if rms else params[per * i + 3], None, None, means[i], rstds[i],
                   ctx.seeds[i:i + 1] if dropped else None, p, dy, None, pres[i], None, dpre,
                   _grad_view(params[per * i + 2]), None if rms else _grad_view(params[per * i + 3]))
            # dW_i += dPre^T X_i: dPre read as stored ([tokens][D] = A^T), X_i as [K = tokens][N = K_i]
            C.gemm_f32x(prec, dpre, True, D, Xs[i], True, K, _grad_view(w), K, K, D, K, N, F32X_ACCUM, None, None)
            C.colsum_f32(dpre, N, D, D, _grad_view(b))
            if i > 0:
                dy = torch.empty((N, K), device=dh.device, dtype=torch.float32)
                C.gemm_f32x(prec, dpre, False, D, w, True, K, dy, K, K, N, K, D, 0, None, None)
            grad_ready(w.grad, b.grad)
        return (None,) * (8 + len(params))


def mlp_encode(x: Tensor, params: Sequence[Tensor], seeds: Optional[Tensor], num_layers: int, norm: str,
               dropout: float, training: bool, precision: str = "medium") -> Tensor:
    """``precision`` = the matmul precision the trainer resolved (``Trainer._effective_matmul_precision``): "medium"
    (``bf16-mixed``, or an explicit medium) runs the bf16 HIP kernels; "high" / "highest" (``32-true``) the fp32 HIP
    path (:class:`_MlpEncoderF32Fn`: bf16x3 / exact-f32 MFMA GEMMs, fp32 norms) -- the trainer's precision is
    honoured, never silently lowered.  ``MTA_EXTRAS_F32_TORCH=1`` keeps the fp32 PyTorch graph for 32-true."""
    if use_hip(x) and precision == "medium":
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        return _MlpEncoderFn.apply(x.contiguous(), seeds, num_layers, norm, float(dropout), bool(training),
                                   need_grad, 0, *params)
    if use_hip(x) and precision in _F32_PREC and not _F32_TORCH:
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        return _MlpEncoderF32Fn.apply(x.contiguous().float(), seeds, num_layers, norm, float(dropout), bool(training),
                                      need_grad, _F32_PREC[precision], *params)
    return mlp_reference(x, params, num_layers, norm, dropout, training)


def mlp_heads_fusable(x: Tensor, params: Sequence[Tensor], num_layers: int, norm: str, precision: str) -> bool:
    """Whether :func:`mlp_encode_heads` fuses the alpha / beta heads into the last norm (bf16 HIP path, last width
    taking the GELU-on-load wide kernels)."""
    per = 4 if norm == "layernorm" else 3
    return (use_hip(x) and precision == "medium" and num_layers >= 1
            and _gelu_in_norm(int(params[per * (num_layers - 1)].shape[0])))


def mlp_encode_heads(x: Tensor, params: Sequence[Tensor], seeds: Optional[Tensor], num_layers: int, norm: str,
                     dropout: float, training: bool, precision: str, heads: Sequence[Tensor]) -> Tensor:
    """``[alpha | beta]`` (N, 2) of the MLP encoder followed by the two Linear(H, 1) heads (``heads`` = (wa (1, H),
    ba (1,), wb, bb)): fused into the last norm kernels when :func:`mlp_heads_fusable`, else encoder + addmm."""
    if mlp_heads_fusable(x, params, num_layers, norm, precision):
        all_p = list(params) + list(heads)
        need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in all_p)
        return _MlpEncoderFn.apply(x.contiguous(), seeds, num_layers, norm, float(dropout), bool(training),
                                   need_grad, 4, *all_p)
    h = mlp_encode(x, params, seeds, num_layers, norm, dropout, training, precision)
    wa, ba, wb, bb = heads
    return torch.addmm(torch.cat([ba, bb]), h, torch.cat([wa, wb], 0).t())


_F32_TORCH = os.environ.get("MTA_EXTRAS_F32_TORCH", "0") == "1"


# --------------------------------------------------------------------------------------------------
# transformer encoder (pre-norm, RMSNorm, RoPE attention, GELU MLP, last-token pooling)
# --------------------------------------------------------------------------------------------------
def rope_reference(x: Tensor, base: float = ROPE_BASE) -> Tensor:
    """Interleaved-pair rotary embedding over (..., T, hd)."""
    T, hd = x.shape[-2], x.shape[-1]
    inv = base ** (-torch.arange(0, hd, 2, device=x.device, dtype=torch.float32) / hd)
    ang = torch.arange(T, device=x.device, dtype=torch.float32)[:, None] * inv[None, :]
    c, s = ang.cos().to(x.dtype), ang.sin().to(x.dtype)
    x0, x1 = x[..., 0::2], x[..., 1::2]
    out = torch.stack([x0 * c - x1 * s, x0 * s + x1 * c], dim=-1)
    return out.flatten(-2)


def attention_reference(qkv: Tensor, heads: int) -> Tensor:
    """qkv (N, T, 3d) -> (N, T, d); RoPE on q, k; bidirectional softmax attention."""
    N, T, d3 = qkv.shape
    d = d3 // 3
    hd = d // heads
    q, k, v = qkv.split(d, dim=-1)
    q = rope_reference(q.view(N, T, heads, hd).transpose(1, 2))
    k = rope_reference(k.view(N, T, heads, hd).transpose(1, 2))
    v = v.view(N, T, heads, hd).transpose(1, 2)
    att = torch.softmax((q @ k.transpose(-1, -2)) / math.sqrt(hd), dim=-1)
    return (att @ v).transpose(1, 2).reshape(N, T, d)


PER_BLOCK = 8  # norm1.w, qkv.w, qkv.b, proj.w, proj.b, norm2.w, fc1.w, fc1.b, fc2.w, fc2.b -> see names below
BLOCK_NAMES = ("norm1.weight", "qkv.weight", "qkv.bias", "proj.weight", "proj.bias", "norm2.weight", "fc1.weight",
               "fc1.bias", "fc2.weight", "fc2.bias")


def transformer_reference(x: Tensor, params: Sequence[Tensor], num_layers: int, heads: int, dropout: float,
                          training: bool) -> Tensor:
    we, be = params[0], params[1]
    h = Fn.linear(x, we, be)
    nb = len(BLOCK_NAMES)
    for l in range(num_layers):
        g1, wqkv, bqkv, wo, bo, g2, w1, b1, w2, b2 = params[2 + nb * l: 2 + nb * (l + 1)]
        a = attention_reference(Fn.linear(Fn.rms_norm(h, (h.shape[-1],), g1, RMS_EPS), wqkv, bqkv), heads)
        h = h + Fn.linear(a, wo, bo)
        u = Fn.gelu(Fn.linear(Fn.rms_norm(h, (h.shape[-1],), g2, RMS_EPS), w1, b1))
        if dropout > 0 and training:
            u = Fn.dropout(u, dropout, True)
        h = h + Fn.linear(u, w2, b2)
    gf = params[2 + nb * num_layers]
    return Fn.rms_norm(h[:, -1], (h.shape[-1],), gf, RMS_EPS)


# fused FFN half of the block (csrc/tr_ffn.hip) for d = 128, dff = 512: RMSNorm2 + FFN-up + GELU + dropout + FFN-down +
# residual in one launch forward, the input-gradient chain + RMSNorm2 backward in one launch backward (its gain gradient
# through f32 atomics, so deterministic mode keeps the unfused chain).  MTA_TR_FFN=0 keeps the unfused chain (A/B).
_TR_FFN = [os.environ.get("MTA_TR_FFN", "1") != "0"]


def set_transformer_ffn_fused(on: bool) -> None:
    _TR_FFN[0] = bool(on)


def _tr_ffn_ok(d: int, dff: int) -> bool:
    return _TR_FFN[0] and not _DETERMINISTIC[0] and d == 128 and dff == 512


# fused attention half of the block forward (csrc/tr_attn.hip) for d = 128, 4 heads, T <= 64: RMSNorm1 + QKV + RoPE +
# attention + projection + residual in one launch, saving exactly the unfused chain's tensors.  MTA_TR_ATTN=0 keeps
# the unfused chain (A/B: transformer_encoder B=1 0.647 -> 0.6175 ms, profiles/r4_transformer_fused_ab.jsonl).
_TR_ATTN = [os.environ.get("MTA_TR_ATTN", "1") != "0"]


def set_transformer_attn_fused(on: bool) -> None:
    _TR_ATTN[0] = bool(on)


# FFN weight gradients as k-contiguous (NN) products: the fused FFN kernels also write u^T, xn2^T (forward) and
# dpre^T, dX^T (backward) as [features][tokens] images, so dW2 += dX^T u and dW1 += dpre^T xn2 read both operands
# along K instead of through the transposed (AT/BT) loaders (0.6175 -> 0.6145 ms; MTA_TR_WGRAD_NN=0 for the A/B).
_TR_WGRAD_NN = [os.environ.get("MTA_TR_WGRAD_NN", "1") != "0"]


def set_transformer_wgrad_nn(on: bool) -> None:
    _TR_WGRAD_NN[0] = bool(on)


def _tr_attn_ok(d: int, heads: int, T: int) -> bool:
    return _TR_ATTN[0] and d == 128 and heads == 4 and 1 <= T <= 64


class _TransformerEncoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, seeds, num_layers, heads, dropout, training, need_grad, *params):
        dev = x.device
        N, T, F = x.shape
        Np = _r8(N)
        M = Np * T
        L = num_layers
        nb = len(BLOCK_NAMES)
        d = params[0].shape[0]
        drop = dropout > 0 and training
        Fp = _r8(F)
        C = lib()
        # bf16 operands: input tokens + every matrix (padded along K only where needed)
        Xin = torch.empty((M, Fp), device=dev, dtype=torch.bfloat16)
        mats = [params[0]]
        for l in range(L):
            base = 2 + nb * l
            mats += [params[base + 1], params[base + 3], params[base + 6], params[base + 8]]
        mats_b = [_padded_bf16(w, _r8(w.shape[1])) for w in mats]
        ffn = _tr_ffn_ok(d, mats_b[3].shape[0] if L else 0)
        attn = _tr_attn_ok(d, heads, T)
        # fused halves: their weights go to fragment-major images instead (FFN: W1, W2 for the forward, W2^T, W1^T
        # for the backward; attention: W_qkv, W_o forward, W_o^T for the backward's dO = dX1 W_o fused into the
        # attention backward, W_qkv^T for its d(xn) = dqkv W_qkv fused into the RMSNorm1 backward), so the
        # row-major casts skip them
        cast = [i for i in range(len(mats))
                if not (i > 0 and ((ffn and (i - 1) % 4 >= 2) or (attn and (i - 1) % 4 < 2)))]
        frag, afrag = None, None
        srcs, dsts, trs = [], [], []
        if ffn:
            frag = torch.empty((L, 4, mats[3].shape[0], d), device=dev, dtype=torch.bfloat16)
            for l in range(L):
                w1, w2 = mats[3 + 4 * l], mats[4 + 4 * l]
                srcs += [w1, w2, w2, w1]
                dsts += [frag[l, 0], frag[l, 1], frag[l, 2], frag[l, 3]]
                trs += [False, False, True, True]
        if attn:
            afrag = [torch.empty_like(mats_b[1 + 4 * l + j]) for l in range(L) for j in (0, 1, 1, 0)]
            srcs += [mats[1 + 4 * l + j] for l in range(L) for j in (0, 1, 1, 0)]
            dsts += afrag
            trs += [False, False, True, True] * L
        # the remaining row-major casts (input tokens -- rows of the padded sequences zero-filled -- and whatever
        # matrices the fused halves do not cover) and the dropout-seed advance: riding on the first packing launch
        # when they fit (one launch for all operand preparation), else cast_pad
        csrc = [x.reshape(N * T, F)] + [mats[i] for i in cast]
        cdst = [Xin] + [mats_b[i] for i in cast]
        ride = bool(srcs) and len(csrc) <= 4
        if not ride:
            cast_pad(csrc, cdst, seeds if drop else None)
        for i in range(0, len(srcs), 32):
            first = i == 0 and ride
            C.frag_pack(srcs[i:i + 32], dsts[i:i + 32], trs[i:i + 32], csrc if first else [], cdst if first else [],
                        seeds if (first and drop) else None)
        xs = torch.empty((M, d), device=dev, dtype=torch.float32)
        # the embedding x = in We^T + be: inside the first fused attention half (fp32 FMAs over the F = 3 inputs),
        # else one GEMM
        embed_fused = attn and L > 0
        if not embed_fused:
            gemm(0, Xin, mats_b[0], M, d, Fp, Fp, Fp, flags=EPI_BIAS, bias=params[1], out_f32=xs)
        saved: List[Tensor] = [Xin]
        stats: List[Tensor] = []
        nn = ffn and _TR_WGRAD_NN[0]  # saved xn2 / u are then the transposed images
        for l in range(L):
            base = 2 + nb * l
            g1, bqkv, bo, g2, b1, b2 = (params[base], params[base + 2], params[base + 4], params[base + 5],
                                        params[base + 7], params[base + 9])
            wqkv_b, wo_b, w1_b, w2_b = mats_b[1 + 4 * l: 5 + 4 * l]
            dff = w1_b.shape[0]
            xn = torch.empty((M, d), device=dev, dtype=torch.bfloat16)
            r1 = torch.empty(M, device=dev, dtype=torch.float32)
            qkv = torch.empty((M, 3 * d), device=dev, dtype=torch.bfloat16)
            o = torch.empty((M, d), device=dev, dtype=torch.bfloat16)
            lse = torch.empty(Np * heads * 64, device=dev, dtype=torch.float32)
            x1 = torch.empty((M, d), device=dev, dtype=torch.float32)
            if attn:
                emb = (x.reshape(N * T, F), params[0], params[1]) if (embed_fused and l == 0) else (None, None, None)
                C.tr_attn_fwd(Np, T, heads, RMS_EPS, ROPE_BASE, xs, afrag[4 * l], afrag[4 * l + 1], g1, bqkv, bo, xn, r1, qkv,
                              o, lse, x1, *emb)
            else:
                C.norm(False, xs, d, M, d, True, RMS_EPS, g1, None, xn, None, None, r1, None, 0.0, None, None, None,
                       None, None, None, None)
                gemm(0, xn, wqkv_b, M, 3 * d, d, d, d, flags=EPI_BIAS, bias=bqkv, out_bf16=qkv)
                C.attention(False, qkv, o, lse, None, None, Np, T, d, heads, ROPE_BASE)
                gemm(0, o, wo_b, M, d, d, d, d, flags=EPI_BIAS | EPI_RESID, bias=bo, resid=xs, out_f32=x1)
            xn2 = torch.empty((d, M) if nn else (M, d), device=dev, dtype=torch.bfloat16)
            r2 = torch.empty(M, device=dev, dtype=torch.float32)
            pre1 = torch.empty((M, dff), device=dev, dtype=torch.bfloat16)
            u = torch.empty((dff, M) if nn else (M, dff), device=dev, dtype=torch.bfloat16)
            x2 = torch.empty((M, d), device=dev, dtype=torch.float32)
            if ffn:
                C.tr_ffn_fwd(x1, frag[l, 0], frag[l, 1].view(d, dff), b1, b2, g2, RMS_EPS, seeds[l:l + 1] if drop else None, float(dropout),
                             None if nn else xn2, r2, pre1, None if nn else u, x2, xn2 if nn else None,
                             u if nn else None)
            else:
                C.norm(False, x1, d, M, d, True, RMS_EPS, g2, None, xn2, None, None, r2, None, 0.0, None, None, None,
                       None, None, None, None)
                fl = EPI_BIAS | EPI_GELU | (EPI_DROPOUT if drop else 0)
                gemm(0, xn2, w1_b, M, dff, d, d, d, flags=fl, bias=b1, seed=seeds[l:l + 1] if drop else None,
                     drop_p=float(dropout), aux_pre=pre1, out_bf16=u)
                gemm(0, u, w2_b, M, d, dff, dff, dff, flags=EPI_BIAS | EPI_RESID, bias=b2, resid=x1, out_f32=x2)
            saved += [xs, xn, qkv, o, x1, xn2, pre1, u]
            stats += [r1, lse, r2]
            xs = x2
        gf = params[2 + nb * L]
        h = torch.empty((Np, d), device=dev, dtype=torch.float32)
        rf = torch.empty(Np, device=dev, dtype=torch.float32)
        C.norm(False, xs.view(-1)[(T - 1) * d:], T * d, Np, d, True, RMS_EPS, gf, None, None, h, None, rf, None, 0.0,
               None, None, None, None, None, None, None)
        saved.append(xs)
        stats.append(rf)
        ctx.meta = (N, Np, T, F, Fp, d, L, heads, drop, float(dropout), ffn, nn)
        ctx.params, ctx.mats_b, ctx.seeds, ctx.frag, ctx.afrag = params, mats_b, seeds, frag, afrag
        if need_grad:
            ctx.save_for_backward(*saved)
            ctx.stats = stats
        return h[:N]

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh):
        N, Np, T, F, Fp, d, L, heads, drop, p, ffn, nn = ctx.meta
        afrag = ctx.afrag  # fused attention half: W_o^T / W_qkv^T images for its fused backward GEMMs
        params, mats_b = ctx.params, ctx.mats_b
        saved = ctx.saved_tensors
        stats = ctx.stats
        C = lib()
        dev = dh.device
        M = Np * T
        nb = len(BLOCK_NAMES)
        Xin = saved[0]
        x_final = saved[-1]
        # final RMSNorm over the last-token rows -> residual-stream gradient, fp32 and bf16 (zero elsewhere): both
        # views of one buffer, zeroed by one kernel
        zbuf = torch.empty(M * d * 6, device=dev, dtype=torch.uint8)
        dX = zbuf[:M * d * 4].view(torch.float32).view(M, d)
        dXb = zbuf[M * d * 4:].view(torch.bfloat16).view(M, d)
        C.zero_(zbuf)
        # the N real sequences only (the padded ones have no output gradient): dh is read in place
        dh = dh if (dh.dtype == torch.float32 and dh.is_contiguous()) else dh.float().contiguous()
        gf = params[2 + nb * L]
        try:
            C.norm_defer()
            C.norm(True, x_final.view(-1)[(T - 1) * d:], T * d, N, d, True, RMS_EPS, gf, None, None, None, None,
                   stats[-1], None, 0.0, dh, None, None, dXb.view(-1)[(T - 1) * d:], dX.view(-1)[(T - 1) * d:],
                   _grad_view(gf), None)
            frag = ctx.frag  # fused FFN: W2^T / W1^T fragment-major images, written by the forward's packing launch
            # operands of the weight gradients queued for the grouped launch: alive (and not rewritten) until the flush
            keep: List[Tensor] = []
            for l in range(L - 1, -1, -1):
                base = 2 + nb * l
                g1, wqkv, bqkv, wo, bo, g2, w1, b1, w2, b2 = params[base: base + nb]
                wqkv_b, wo_b, w1_b, w2_b = mats_b[1 + 4 * l: 5 + 4 * l]
                dff = w1_b.shape[0]
                xs, xn, qkv, o, x1, xn2, pre1, u = saved[1 + 8 * l: 9 + 8 * l]
                r1, lse, r2 = stats[3 * l: 3 * l + 3]
                dpre1 = torch.empty((dff, M) if nn else (M, dff), device=dev, dtype=torch.bfloat16)
                dX1 = torch.empty((M, d), device=dev, dtype=torch.float32)
                dX1b = torch.empty((M, d), device=dev, dtype=torch.bfloat16)
                if nn:
                    # same chain; the weight gradients then run on the transposed images as NN products (one paired launch)
                    dXt = torch.empty((d, M), device=dev, dtype=torch.bfloat16)
                    C.tr_ffn_bwd(x1, frag[l, 3].view(d, dff), frag[l, 2], g2, r2, pre1, ctx.seeds[l:l + 1] if drop else None,
                                 p, dX, dXb, None, dX1, dX1b, _grad_view(g2), dpre1, dXt)
                    gemm(0, dXt, u, d, dff, M, M, M, flags=EPI_ACCUM, out_f32=_grad_view(w2), ldc=dff,
                         ksplit=wgrad_split(d, dff, M), bias_grad=_grad_view(b2), group=True)
                    gemm(0, dpre1, xn2, dff, d, M, M, M, flags=EPI_ACCUM, out_f32=_grad_view(w1), ldc=d,
                         ksplit=wgrad_split(dff, d, M), bias_grad=_grad_view(b1), group=True)
                    keep += [dXt, dpre1]
                elif ffn:
                    # d(u) = dX W2 -> dPre1 -> d(xn2) = dPre1 W1 -> dX1 = norm2_bwd(d(xn2)) + dX, one launch; then the
                    # two weight gradients dW2 += dX^T u (db2), dW1 += dPre1^T xn2 (db1)
                    C.tr_ffn_bwd(x1, frag[l, 3].view(d, dff), frag[l, 2], g2, r2, pre1, ctx.seeds[l:l + 1] if drop else None,
                                 p, dX, dXb, dpre1, dX1, dX1b, _grad_view(g2), None, None)
                    gemm(2, dXb, u, d, dff, M, d, dff, flags=EPI_ACCUM, out_f32=_grad_view(w2), ldc=dff,
                         ksplit=wgrad_split(d, dff, M), bias_grad=_grad_view(b2), group=True)
                    gemm(2, dpre1, xn2, dff, d, M, dff, d, flags=EPI_ACCUM, out_f32=_grad_view(w1), ldc=d,
                         ksplit=wgrad_split(dff, d, M), bias_grad=_grad_view(b1), group=True)
                    keep += [dXb, dpre1]
                else:
                    # fc2: dW2 += dX^T u, db2; d(u) -> dPre1 = d(u) * dropout * gelu'(pre1)
                    gemm(2, dXb, u, d, dff, M, d, dff, flags=EPI_ACCUM, out_f32=_grad_view(w2), ldc=dff,
                         ksplit=wgrad_split(d, dff, M), bias_grad=_grad_view(b2), group=True)
                    fl = EPI_DGELU | (EPI_DROPOUT if drop else 0)
                    gemm(1, dXb, w2_b, M, dff, d, d, dff, flags=fl, aux_in=pre1,
                         seed=ctx.seeds[l:l + 1] if drop else None, drop_p=p, out_bf16=dpre1)
                    # fc1: dW1 += dPre1^T xn2, db1; d(xn2) = dPre1 W1
                    gemm(2, dpre1, xn2, dff, d, M, dff, d, flags=EPI_ACCUM, out_f32=_grad_view(w1), ldc=d,
                         ksplit=wgrad_split(dff, d, M), bias_grad=_grad_view(b1), group=True)
                    keep += [dXb, dpre1]
                    dxn2 = torch.empty((M, d), device=dev, dtype=torch.float32)
                    gemm(1, dpre1, w1_b, M, d, dff, dff, d, out_f32=dxn2)
                    # RMSNorm2 backward + residual: dX1 = norm2_bwd(dxn2) + dX
                    C.norm_defer()  # dgamma: one batched reduction launch at the end of the backward
                    C.norm(True, x1, d, M, d, True, RMS_EPS, g2, None, None, None, None, r2, None, 0.0, dxn2, dX, None,
                           dX1b, dX1, _grad_view(g2), None)
                # proj: dWo += dX1^T o, dbo; d(o) = dX1 Wo
                gemm(2, dX1b, o, d, d, M, d, d, flags=EPI_ACCUM, out_f32=_grad_view(wo), ldc=d,
                     ksplit=wgrad_split(d, d, M), bias_grad=_grad_view(bo), group=True)
                # attention backward (RoPE inverse fused) -> dqkv; d(o) = dX1 Wo inside it (fused half) or a GEMM before it
                dqkv = torch.empty((M, 3 * d), device=dev, dtype=torch.bfloat16)
                if afrag is not None:
                    C.attention(True, qkv, o, lse, None, dqkv, Np, T, d, heads, ROPE_BASE, dX1b, afrag[4 * l + 2])
                else:
                    do = torch.empty((M, d), device=dev, dtype=torch.bfloat16)
                    gemm(1, dX1b, wo_b, M, d, d, d, d, out_bf16=do)
                    C.attention(True, qkv, o, lse, do, dqkv, Np, T, d, heads, ROPE_BASE)
                # qkv: dWqkv += dqkv^T xn, dbqkv; d(xn) = dqkv Wqkv
                gemm(2, dqkv, xn, 3 * d, d, M, 3 * d, d, flags=EPI_ACCUM, out_f32=_grad_view(wqkv), ldc=d,
                     ksplit=wgrad_split(3 * d, d, M), bias_grad=_grad_view(bqkv), group=True)
                keep += [dX1b, dqkv]
                dXn = torch.empty((M, d), device=dev, dtype=torch.float32)
                dXb = torch.empty((M, d), device=dev, dtype=torch.bfloat16)  # fresh: the queued dW2 may read the last one
                if afrag is not None:
                    # d(xn) = dqkv Wqkv and the RMSNorm1 backward + residual in one launch (dg1: deferred norm slot)
                    C.tr_attn_dx(dqkv, afrag[4 * l + 3], xs, r1, g1, dX1, dXn, dXb, _grad_view(g1))
                else:
                    dxn = torch.empty((M, d), device=dev, dtype=torch.float32)
                    gemm(1, dqkv, wqkv_b, M, d, 3 * d, 3 * d, d, out_f32=dxn)
                    # RMSNorm1 backward + residual: dX = norm1_bwd(dxn) + dX1
                    C.norm_defer()
                    C.norm(True, xs, d, M, d, True, RMS_EPS, g1, None, None, None, None, r1, None, 0.0, dxn, dX1, None,
                           dXb, dXn, _grad_view(g1), None)
                dX = dXn
            # embedding: dWe += dX^T Xin (F real columns of Fp), dbe
            gemm(2, dXb, Xin, d, Fp, M, d, Fp, flags=EPI_ACCUM, out_f32=_grad_view(params[0]), ldc=F, n_store=F,
                 ksplit=wgrad_split(d, Fp, M), bias_grad=_grad_view(params[1]), group=True)
            # every layer's weight gradients in one launch per operand layout (queued above), then the norm gains
            gemm_group_flush()
            del keep
            C.norm_flush()
        except BaseException:
            # the queued weight gradients hold raw pointers to operands only ``keep`` keeps alive, and the deferred
            # norm slots may be unwritten: drop both so the next flush cannot launch them on freed memory
            C.gemm_group_discard()
            C.norm_discard()
            raise
        for l in range(L):
            base = 2 + nb * l
            grad_ready(*(params[base + j].grad for j in (1, 2, 3, 4, 6, 7, 8, 9)))
        return (None,) * (7 + len(params))


# --------------------------------------------------------------------------------------------------
# 32-true transformer encoder on HIP kernels: every tensor fp32, the seven GEMMs of a block on gemm_f32x at the
# resolved matmul precision (bf16x3 / exact f32) with bias, GELU (input saved), dropout (counter hash), GELU' and the
# residual add fused into their epilogues; RMSNorm forward / backward (residual-stream gradient fused) on norm.hip;
# RoPE attention forward / backward in fp32 on attention_f32.hip.  Reference math: transformer_reference.
# --------------------------------------------------------------------------------------------------
def _tr_f32_ok(d: int, heads: int, T: int) -> bool:
    """Shapes the fp32 attention kernel covers: T <= 64, head dim 16 / 32 / 64 (the fp32 LDS image of one (sequence,
    head) problem)."""
    return 1 <= T <= 64 and heads >= 1 and d % heads == 0 and d // heads in (16, 32, 64)


class _TransformerEncoderF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, seeds, num_layers, heads, dropout, training, need_grad, prec, *params):
        dev = x.device
        N, T, F = x.shape
        M = N * T
        L = num_layers
        nb = len(BLOCK_NAMES)
        d = params[0].shape[0]
        drop = dropout > 0 and training
        C = lib()
        if drop:
            C.seeds_advance(seeds)
        f32 = dict(device=dev, dtype=torch.float32)
        X0 = x.reshape(M, F)
        xs = torch.empty((M, d), **f32)
        C.gemm_f32x(prec, X0, False, F, params[0], False, F, xs, d, d, M, d, F, F32X_BIAS, params[1], None)
        saved: List[Tensor] = [X0]
        stats: List[Tensor] = []
        for l in range(L):
            g1, wqkv, bqkv, wo, bo, g2, w1, b1, w2, b2 = params[2 + nb * l: 2 + nb * (l + 1)]
            dff = w1.shape[0]
            xn, r1 = torch.empty((M, d), **f32), torch.empty(M, **f32)
            C.norm(False, xs, d, M, d, True, RMS_EPS, g1, None, None, xn, None, r1, None, 0.0, None, None, None, None,
                   None, None, None)
            qkv = torch.empty((M, 3 * d), **f32)
            C.gemm_f32x(prec, xn, False, d, wqkv, False, d, qkv, 3 * d, 3 * d, M, 3 * d, d, F32X_BIAS, bqkv, None)
            o, lse = torch.empty((M, d), **f32), torch.empty(N * heads * 64, **f32)
            C.attention_f32(False, qkv, o, lse, None, None, N, T, d, heads, ROPE_BASE)
            x1 = torch.empty((M, d), **f32)
            C.gemm_f32x(prec, o, False, d, wo, False, d, x1, d, d, M, d, d, F32X_BIAS | F32X_RESID, bo, None,
                        resid=xs)
            xn2, r2 = torch.empty((M, d), **f32), torch.empty(M, **f32)
            C.norm(False, x1, d, M, d, True, RMS_EPS, g2, None, None, xn2, None, r2, None, 0.0, None, None, None, None,
                   None, None, None)
            pre1, u = torch.empty((M, dff), **f32), torch.empty((M, dff), **f32)
            C.gemm_f32x(prec, xn2, False, d, w1, False, d, u, dff, dff, M, dff, d,
                        F32X_BIAS | F32X_GELU | (F32X_DROPOUT if drop else 0), b1, pre1,
                        seed=seeds[l:l + 1] if drop else None, drop_p=float(dropout) if drop else 0.0)
            x2 = torch.empty((M, d), **f32)
            C.gemm_f32x(prec, u, False, dff, w2, False, dff, x2, d, d, M, d, dff, F32X_BIAS | F32X_RESID, b2, None,
                        resid=x1)
            saved += [xs, xn, qkv, o, x1, xn2, pre1, u]
            stats += [r1, lse, r2]
            xs = x2
        gf = params[2 + nb * L]
        h, rf = torch.empty((N, d), **f32), torch.empty(N, **f32)
        # final RMSNorm on the last token of each sequence: rows T*d apart
        C.norm(False, xs.view(-1)[(T - 1) * d:], T * d, N, d, True, RMS_EPS, gf, None, None, h, None, rf, None, 0.0,
               None, None, None, None, None, None, None)
        saved.append(xs)
        stats.append(rf)
        ctx.meta = (N, T, F, d, L, heads, drop, float(dropout), prec)
        ctx.params, ctx.seeds = params, seeds
        if need_grad:
            ctx.save_for_backward(*saved)
            ctx.stats = stats
        return h

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh):
        N, T, F, d, L, heads, drop, p, prec = ctx.meta
        params = ctx.params
        saved = ctx.saved_tensors
        stats = ctx.stats
        C = lib()
        M = N * T
        nb = len(BLOCK_NAMES)
        f32 = dict(device=dh.device, dtype=torch.float32)
        dh = dh if (dh.dtype == torch.float32 and dh.is_contiguous()) else dh.float().contiguous()
        # final RMSNorm backward -> residual-stream gradient on the last-token rows (zero elsewhere)
        dX = torch.empty((M, d), **f32)
        C.zero_(dX)
        gf = params[2 + nb * L]
        C.norm(True, saved[-1].view(-1)[(T - 1) * d:], T * d, N, d, True, RMS_EPS, gf, None, None, None, None,
               stats[-1], None, 0.0, dh, None, None, None, dX.view(-1)[(T - 1) * d:], _grad_view(gf), None)
        for l in range(L - 1, -1, -1):
            g1, wqkv, bqkv, wo, bo, g2, w1, b1, w2, b2 = params[2 + nb * l: 2 + nb * (l + 1)]
            dff = w1.shape[0]
            xs, xn, qkv, o, x1, xn2, pre1, u = saved[1 + 8 * l: 9 + 8 * l]
            r1, lse, r2 = stats[3 * l: 3 * l + 3]
            # fc2: dW2 += dX^T u, db2; dPre1 = (dX W2) * dropout * GELU'(pre1)
            C.gemm_f32x(prec, dX, True, d, u, True, dff, _grad_view(w2), dff, dff, d, dff, M, F32X_ACCUM, None, None)
            C.colsum_f32(dX, M, d, d, _grad_view(b2))
            dpre1 = torch.empty((M, dff), **f32)
            C.gemm_f32x(prec, dX, False, d, w2, True, dff, dpre1, dff, dff, M, dff, d,
                        F32X_DGELU | (F32X_DROPOUT if drop else 0), None, pre1,
                        seed=ctx.seeds[l:l + 1] if drop else None, drop_p=p if drop else 0.0)
            # fc1: dW1 += dPre1^T xn2, db1; d(xn2) = dPre1 W1
            C.gemm_f32x(prec, dpre1, True, dff, xn2, True, d, _grad_view(w1), d, d, dff, d, M, F32X_ACCUM, None,
                        None)
            C.colsum_f32(dpre1, M, dff, dff, _grad_view(b1))
            dxn2 = torch.empty((M, d), **f32)
            C.gemm_f32x(prec, dpre1, False, dff, w1, True, d, dxn2, d, d, M, d, dff, 0, None, None)
            # RMSNorm2 backward + residual: dX1 = norm2_bwd(dxn2) + dX
            dX1 = torch.empty((M, d), **f32)
            C.norm(True, x1, d, M, d, True, RMS_EPS, g2, None, None, None, None, r2, None, 0.0, dxn2, dX, None, None,
                   dX1, _grad_view(g2), None)
            # proj: dWo += dX1^T o, dbo; d(o) = dX1 Wo
            C.gemm_f32x(prec, dX1, True, d, o, True, d, _grad_view(wo), d, d, d, d, M, F32X_ACCUM, None, None)
            C.colsum_f32(dX1, M, d, d, _grad_view(bo))
            do = torch.empty((M, d), **f32)
            C.gemm_f32x(prec, dX1, False, d, wo, True, d, do, d, d, M, d, d, 0, None, None)
            # attention backward (inverse RoPE fused) -> dqkv
            dqkv = torch.empty((M, 3 * d), **f32)
            C.attention_f32(True, qkv, o, lse, do, dqkv, N, T, d, heads, ROPE_BASE)
            # qkv: dWqkv += dqkv^T xn, dbqkv; d(xn) = dqkv Wqkv
            C.gemm_f32x(prec, dqkv, True, 3 * d, xn, True, d, _grad_view(wqkv), d, d, 3 * d, d, M, F32X_ACCUM, None,
                        None)
            C.colsum_f32(dqkv, M, 3 * d, 3 * d, _grad_view(bqkv))
            dxn = torch.empty((M, d), **f32)
            C.gemm_f32x(prec, dqkv, False, 3 * d, wqkv, True, d, dxn, d, d, M, d, 3 * d, 0, None, None)
            grad_ready(wqkv.grad, bqkv.grad, wo.grad, bo.grad, w1.grad, b1.grad, w2.grad, b2.grad)
            # RMSNorm1 backward + residual: dX = norm1_bwd(dxn) + dX1
            dXn = torch.empty((M, d), **f32)
            C.norm(True, xs, d, M, d, True, RMS_EPS, g1, None, None, None, None, r1, None, 0.0, dxn, dX1, None, None,
                   dXn, _grad_view(g1), None)
            dX = dXn
        # embedding: dWe += dX^T X0, dbe
        C.gemm_f32x(prec, dX, True, d, saved[0], True, F, _grad_view(params[0]), F, F, d, F, M, F32X_ACCUM, None,
                    None)
        C.colsum_f32(dX, M, d, d, _grad_view(params[1]))
        return (None,) * (8 + len(params))


def transformer_encode(x: Tensor, params: Sequence[Tensor], seeds: Optional[Tensor], num_layers: int, heads: int,
                       dropout: float, training: bool, precision: str = "medium") -> Tensor:
    """``precision``: as :func:`mlp_encode` ("high" / "highest": :class:`_TransformerEncoderF32Fn` when the fp32
    attention kernel covers the shape, else the fp32 PyTorch graph)."""
    need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
    if use_hip(x) and precision == "medium":
        return _TransformerEncoderFn.apply(x.contiguous(), seeds, num_layers, heads, float(dropout), bool(training),
                                           need_grad, *params)
    if (use_hip(x) and precision in _F32_PREC and not _F32_TORCH
            and _tr_f32_ok(params[0].shape[0], heads, x.shape[1])):
        return _TransformerEncoderF32Fn.apply(x.contiguous().float(), seeds, num_layers, heads, float(dropout),
                                              bool(training), need_grad, _F32_PREC[precision], *params)
    return transformer_reference(x, params, num_layers, heads, dropout, training)
