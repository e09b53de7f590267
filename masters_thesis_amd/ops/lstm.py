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

from typing import List, Optional, Sequence

import os

import torch
from torch import Tensor

from ._lib import lib, use_hip

# torch.set_float32_matmul_precision names -> csrc/common.h PREC_* codes.  "high" is PyTorch's TF32-class setting
# (TF32, or bf16x2/x3 sums): here the LSTM forward's recurrent / input products run PREC_F16X2 (fp16 activations,
# fp16 hi + lo weights: 2 MFMA passes, r4 probe fwd 87 -> 80 us at the headline shape, profiles/r4_lstm_f16x2_ab.txt)
# and every backward product bf16x3.  "bf16x3" forces the r3 form (3 bf16 passes forward too); so does
# MTA_LSTM_HIGH=bf16x3 for "high".
MATMUL_PRECISION = {"highest": 0, "high": 3, "medium": 2, "bf16x3": 1, "f16x2": 3}
if os.environ.get("MTA_LSTM_HIGH", "") == "bf16x3":
    MATMUL_PRECISION["high"] = 1
# deterministic mode (Trainer(deterministic=True)): the weight-gradient chunks write partials that are summed
# in chunk order by one extra launch instead of f32 atomics, so two runs are bit-identical
_DETERMINISTIC = [False]


def set_deterministic(flag: bool) -> None:
    _DETERMINISTIC[0] = bool(flag)


def _parts(C, fused: bool, T: int, H: int, fins, device):
    if not _DETERMINISTIC[0]:
        return []
    return [torch.empty(C.lstm_wgrad_part_floats(int(fused), T, H, f), device=device, dtype=torch.float32)
            for f in fins]
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
                # time-parallel input projection on the MFMA GEMM at the op's precision (csrc/gemm_f32.hip)
                inp = inp.contiguous()
                gx = torch.empty((T * Np, 4 * H), device=dev, dtype=torch.float32)
                C.gemm_f32(prec, inp, w_um, gx, b_um, None, False)
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
            part = _parts(C, False, T, H, [inp.shape[-1]], dG.device)
            C.lstm_wgrad(ctx.prec, dG, hseq, inp, fused0, N, Np, T, H, _grad_buffer(w_ih), _grad_buffer(w_hh),
                         _grad_buffer(b_ih), _grad_buffer(b_hh), part[0] if part else None)
            dG2 = dG.view(T * Np, 4 * H)
            if l > 0:
                # dx = dG W_ih (x the input-dropout mask in the epilogue); W_um is [4H][H] = [K][N]
                dinp = torch.empty((T * Np, H), device=dG.device, dtype=torch.float32)
                C.gemm_f32(ctx.prec, dG2, w_um, dinp, None,
                           masks[l - 1] if ctx.dropout > 0.0 and ctx.training else None, True)
                dH = dinp.view(T, Np, H)
            elif ctx.needs_input_grad[0]:
                perm = _unit_major_rows(H, dG.device)
                w_sel = w_ih.index_select(0, perm).contiguous()
                dx = torch.empty((T * Np, F), device=dG.device, dtype=torch.float32)
                C.gemm_f32(ctx.prec, dG2, w_sel, dx, None, None, True)
                dx = dx.view(T, Np, F)[:, :N].transpose(0, 1)
        return (dx, None, None, None, None, *([None] * (4 * L)))


_E = {}


def _empty(dev, dtype=torch.float32) -> Tensor:
    key = (str(dev), dtype)
    if key not in _E:
        _E[key] = torch.empty(0, device=dev, dtype=dtype)
    return _E[key]


def pipeline_supported(x: Tensor, weights: Sequence[Tensor], num_layers: int) -> bool:
    """Layer-pipelined single-launch path (csrc/lstm_stack.hip) applicability."""
    import os

    if os.environ.get("MTA_LSTM_PIPELINE", "1") == "0" or x.requires_grad:
        return False
    H = weights[1].shape[1]
    N, T, F = x.shape
    # No co-residency cap: a hand-off's producer workgroup always has a lower block id than its consumers
    # (layer-major ids; the backward lists the top layer first), so with in-order dispatch every resident
    # spinning workgroup's producers are resident or finished.  Grids beyond one workgroup per CU (large
    # batches: B=64 is 800 workgroups) run in waves instead of falling back to per-layer launches and
    # T x Np x 4H gate tensors.
    # long sequences: progress words carry more step bits (csrc/lstm_stack.hip epoch_shift), the stash is O(T)
    # (T = 100k, N = 100, H = 64: 14 GB per layer of 288 GB HBM)
    return (H in (32, 64) or 8 <= H < 32) and F in FUSED_F and 1 <= num_layers <= 8 and T + 8 < (1 << 22)


_FLAGS = {}
_CTL_WORDS = 160  # control words at the end of the flag buffer (csrc/lstm_stack.hip CTL_*): [0] = timeout count


def _stack_flags(C, Np: int, L: int, device, T: int = 60) -> Tensor:
    """Persistent, zero-initialised progress/epoch words of the pipelined kernels (never reset per launch:
    progress is epoch-stamped in-kernel, so a captured graph has no memset nodes).

    One buffer per (Np, L, device): every progress word a launch polls is then rewritten by every launch
    that shares the buffer, so a stale word is always exactly one epoch behind and compares below the
    awaited value under the kernel's wrap-safe signed difference.  (A buffer shared between stack depths
    would leave the deeper layers' words at 0 while the epoch advances; once the epoch passes 2^19 such a
    never-written word would read as 'reached'.)  The key includes the progress words' epoch shift (a function
    of T): words written under one shift are never compared under another."""
    key = (C.lstm_stack_flag_words(Np), int(L), str(device), int(C.lstm_stack_epoch_shift(int(T))))
    if key not in _FLAGS:
        _FLAGS[key] = torch.zeros(key[0], dtype=torch.int32, device=device)
    return _FLAGS[key]


_GRAN = {}
# the decoupled forward wins up to B = 4 windows and loses from B = 8 on (probe, L = 2: N = 200 72.9 vs 81.3 us,
# 400 73.8 vs 81.1, 800 85.0 vs 83.8, 1,600 102.7 vs 98.3, 6,400 610 vs 447; profiles/r6_lstm_dec/r6w_probe.txt):
# its input waves' x-image work outweighs the barrier it saves once several tiles share a CU
DEC_MAX_NP = 512


def _stack_gran(C, Np: int, L: int, device, T: int, H: int) -> Optional[Tensor]:
    """Hand-off granules of the decoupled forward (csrc/lstm_stack.hip stack_fwd_dec): layer l >= 1's input as
    {value, epoch-stamped step} pairs, int64 (L - 1, T, Np, H).  None selects the barrier form (``MTA_LSTM_DEC=0``).

    Tags carry the forward epoch of the flag buffer (``_stack_flags``), so the granule buffer is keyed like it (plus
    T and H): every launch that writes it draws its epoch from that one buffer, and a stale granule always carries an
    older epoch than the one a launch waits for."""
    import os

    if os.environ.get("MTA_LSTM_DEC", "1") == "0" or Np > DEC_MAX_NP:
        return None
    key = (C.lstm_stack_flag_words(Np), int(Np), int(L), str(device), int(C.lstm_stack_epoch_shift(int(T))), int(T),
           int(H))
    if key not in _GRAN:
        _GRAN[key] = torch.zeros(max(L - 1, 1) * T * Np * H, dtype=torch.int64, device=device)
    return _GRAN[key]


def stack_timeouts(flags: Tensor) -> int:
    """Number of hand-off waits that gave up since the last check (host sync)."""
    return int(flags[flags.numel() - _CTL_WORDS].item())


def check_pipeline_health(clear: bool = True) -> None:
    """Raise if any pipelined LSTM launch gave up waiting on a producer (its outputs were garbage).

    The kernels bound every spin (the grid always drains) and count give-ups in a device word; the
    trainer calls this at every epoch end and ``bench.py`` after its timed loop."""
    bad = []
    for (words, L, dev, _shift), f in _FLAGS.items():
        n = stack_timeouts(f)
        if n:
            bad.append(f"L={L} on {dev}: {n} wait(s)")
            if clear:
                f[f.numel() - _CTL_WORDS].zero_()
    if bad:
        raise RuntimeError("pipelined LSTM hand-off timed out (results of the affected steps are invalid): "
                           + "; ".join(bad) + ". Another process time-slicing the GPU, or MTA_LSTM_SPIN_LIMIT "
                           "set too low, can cause this; MTA_LSTM_PIPELINE=0 selects the per-layer kernels.")


class PipelinedState:
    """What the pipelined backward needs from its forward (the autograd Function's ctx, or held by the
    trainer's fused step)."""
    __slots__ = ("meta", "params", "seeds", "x", "stash", "hseq", "xdrop", "masks", "pad")


def _padded_rows_index(H: int, Hp: int, device) -> Tensor:
    """nn.LSTM gate row g*H + u of an H-unit layer -> row g*Hp + u of the zero-padded Hp-unit layer."""
    return (torch.arange(4, device=device)[:, None] * Hp + torch.arange(H, device=device)[None, :]).reshape(-1)


def _pad_weights(flat: Sequence[Tensor], H: int, Hp: int, F: int) -> List[Tensor]:
    """Zero-pad an H-unit stack to Hp units.  Exact: a padded unit has zero weights and bias, so its gates are
    (0.5, 0.5, 0, 0.5), its c stays 0 and its h is exactly 0; its outgoing weights are zero too, so it never
    reaches a real unit, and every gradient of a padding weight is exactly 0 (the thesis grid's H=16 runs
    on the H=32 kernels: SURVEY A.2, `tex/diplomski_rad.tex:1106-1122`)."""
    idx = _padded_rows_index(H, Hp, flat[0].device)
    out = []
    for l in range(len(flat) // 4):
        w_ih, w_hh, b_ih, b_hh = flat[4 * l: 4 * l + 4]
        fin = F if l == 0 else H
        fin_p = F if l == 0 else Hp
        pw = w_ih.new_zeros((4 * Hp, fin_p))
        pw[:, :fin].index_copy_(0, idx, w_ih.detach())
        ph = w_hh.new_zeros((4 * Hp, Hp))
        ph[:, :H].index_copy_(0, idx, w_hh.detach())
        out += [pw, ph, b_ih.new_zeros(4 * Hp).index_copy_(0, idx, b_ih.detach()),
                b_hh.new_zeros(4 * Hp).index_copy_(0, idx, b_hh.detach())]
    return out


def kernel_hidden(H: int) -> int:
    """Hidden size the pipelined kernels run an H-unit stack at (native 32 / 64; H < 32 zero-padded to 32)."""
    return H if H in (32, 64) else 32


def pipelined_forward(x: Tensor, seeds: Tensor, prec: int, dropout: float, training: bool, need_grad: bool,
                      flat: Sequence[Tensor], gather=None):
    """One forward launch of every layer (csrc/lstm_stack.hip).  Returns (h_T of the top layer (N, H), state).

    ``gather`` = (src tensors, static buffers, perm, cursor, B) of a deferred static batch
    (data/loaders.py DeferredBatch): the launch reads x through the permutation and fills the buffers itself
    (``x`` must be the static x buffer, viewed (B*K, T, F))."""
    L = len(flat) // 4
    N, T, F = x.shape
    H0 = flat[1].shape[1]
    H = kernel_hidden(H0)
    pad = None
    if H != H0:
        pad = (tuple(flat), H0)
        flat = _pad_weights(flat, H0, H, F)
    Np = padded_rows(N)
    C = lib()
    dev = x.device
    E = _empty(dev)
    drop = dropout > 0.0 and training
    if drop and not need_grad:
        # the backward launch advances the seeds after use; without one, advance them here
        seeds.add_(0x9E3779B97F4A7C15 - (1 << 64))
    hseq = [torch.empty((T, Np, H), device=dev, dtype=torch.float32) for _ in range(L)]
    xdrop = [E] + [torch.empty((T, Np, H), device=dev, dtype=torch.float32) if drop else E for _ in range(1, L)]
    EB = _empty(dev, torch.uint8)
    # keep bytes of every inter-layer dropout, drawn by the forward's input waves and read by the backward's
    # dx keep bytes (u32 words (T, ntiles, 16, H/4): byte e of word (t, tile, s, c) = unit 4c+e of sequence s)
    masks = [EB] + [torch.empty((T, Np, H), device=dev, dtype=torch.uint8) if drop else EB for _ in range(1, L)]
    stash = [torch.empty(T * Np * 5 * H, device=dev, dtype=torch.float32) if need_grad else E for _ in range(L)]
    flags = _stack_flags(C, Np, L, dev, T)
    gran = _stack_gran(C, Np, L, dev, T, H)
    if gather is not None:
        src, dst, perm, cursor, B = gather
        if x.data_ptr() != dst[0].data_ptr() or not x.is_contiguous():
            raise ValueError("deferred gather: x must be the static batch buffer")
        C.lstm_stack_fwd_gather(H, prec, F, x, list(flat[0::4]), list(flat[1::4]), list(flat[2::4]),
                                list(flat[3::4]), hseq, xdrop, masks, stash, seeds, float(dropout), flags, N, Np, T,
                                src, dst, perm, cursor, B, gran)
    else:
        C.lstm_stack_fwd(H, prec, F, x, list(flat[0::4]), list(flat[1::4]), list(flat[2::4]), list(flat[3::4]),
                         hseq, xdrop, masks, stash, seeds, float(dropout), flags, N, Np, T, gran)
    st = PipelinedState()
    st.meta = (L, H, N, Np, T, F, prec, float(dropout), drop)
    st.params, st.seeds, st.x = tuple(flat), seeds, x
    st.stash, st.hseq, st.xdrop, st.masks = stash, hseq, xdrop, masks
    st.pad = pad
    if pad is not None:
        return hseq[L - 1][T - 1, :N, :H0], st
    return hseq[L - 1][T - 1, :N], st


def pipelined_backward(st: "PipelinedState", dh_last: Tensor) -> None:
    """One backward launch (BPTT of every layer + fused weight gradients accumulated into the parameters'
    ``.grad`` views)."""
    L, H, N, Np, T, F, prec, p, drop = st.meta
    C = lib()
    dev = dh_last.device
    flat = st.params
    if st.pad is not None:  # zero-padded stack: pad dh, accumulate into padded buffers, scatter back below
        H0 = st.pad[1]
        dh_p = dh_last.new_zeros((N, H))
        dh_p[:, :H0] = dh_last
        dh_last = dh_p
        for t in flat:
            t.grad = torch.zeros_like(t)
    dG = [torch.empty((T, Np, 4 * H), device=dev, dtype=torch.float32) for _ in range(L)]
    # dX hand-off between layers: fp32 rows + progress words (form 0).  The kernel keeps a tagged-granule form
    # (form 1, A/B only: slower at every depth, profiles/r6_lstm_decoupled.txt)
    form = 0
    dX = [torch.empty((T, Np, H), device=dev, dtype=torch.float32) for _ in range(L - 1)] + [_empty(dev)]
    flags = _stack_flags(C, Np, L, dev, T)
    inp = [st.x] + [st.xdrop[l] if drop else st.hseq[l - 1] for l in range(1, L)]
    grads = [[_grad_buffer(flat[4 * l + k]) for l in range(L)] for k in range(4)]
    parts = _parts(C, True, T, H, [F] + [H] * (L - 1), dev)
    C.lstm_stack_bwd(H, prec, F, list(st.stash), list(flat[1::4]), list(flat[0::4]), dh_last.contiguous(), dG, dX,
                     list(st.hseq), inp, grads, list(st.masks) if drop else [], parts, st.seeds, p, drop, flags, N,
                     Np, T, form)
    if st.pad is not None:
        real, H0 = st.pad
        idx = _padded_rows_index(H0, H, dev)
        for l in range(L):
            fin = F if l == 0 else H0
            pw, ph, pbi, pbh = flat[4 * l: 4 * l + 4]
            w_ih, w_hh, b_ih, b_hh = real[4 * l: 4 * l + 4]
            _grad_buffer(w_ih).add_(pw.grad.index_select(0, idx)[:, :fin])
            _grad_buffer(w_hh).add_(ph.grad.index_select(0, idx)[:, :H0])
            _grad_buffer(b_ih).add_(pbi.grad.index_select(0, idx))
            _grad_buffer(b_hh).add_(pbh.grad.index_select(0, idx))


class _LSTMPipelinedFn(torch.autograd.Function):
    """All layers in one forward launch and one backward launch (wavefront over (layer, t))."""

    @staticmethod
    def forward(ctx, x: Tensor, seeds: Tensor, prec: int, dropout: float, training: bool, need_grad: bool,
                *flat: Tensor) -> Tensor:
        out, st = pipelined_forward(x, seeds, prec, dropout, training, need_grad, flat)
        ctx.st = st
        return out

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, dh_last: Tensor):
        pipelined_backward(ctx.st, dh_last)
        ctx.st = None
        return (None,) * len(ctx.needs_input_grad)


_PERM_CACHE = {}


def _unit_major_rows(H: int, device) -> Tensor:
    """perm[c'] = r for unit-major gate column c' = 4u + g and nn.LSTM row r = g*H + u."""
    key = (H, str(device))
    if key not in _PERM_CACHE:
        c = torch.arange(4 * H)
        _PERM_CACHE[key] = ((c % 4) * H + c // 4).to(device)
    return _PERM_CACHE[key]


def lstm_last_hidden(x: Tensor, weights: Sequence[Tensor], num_layers: int, dropout: float, training: bool,
                     precision=None, seeds: Tensor = None) -> Tensor:
    """Run the stacked LSTM over batch-first ``x (N, T, F)`` and return ``h_T`` of the top layer (N, H).

    ``weights`` is nn.LSTM's flat list ``[w_ih_l0, w_hh_l0, b_ih_l0, b_hh_l0, w_ih_l1, ...]``.
    ``seeds`` (int64[>= L] on the device) drives the pipelined path's counter-hash dropout masks.
    """
    if use_hip(x) and pipeline_supported(x, weights, num_layers) and (
            seeds is not None or not (dropout > 0 and training)):
        if seeds is None:
            seeds = torch.zeros(8, dtype=torch.int64, device=x.device)
        need_grad = torch.is_grad_enabled() and any(t.requires_grad for t in weights)
        return _LSTMPipelinedFn.apply(x.contiguous(), seeds, precision_code(precision), float(dropout),
                                      bool(training), need_grad, *weights)
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
