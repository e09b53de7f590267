"""Timing of the pipelined LSTM stack kernels vs the per-layer kernels (fwd / bwd, L = 1..8).

(The MTA_STACK_PLAIN_STORES probes of round 1 showed the stash traffic costing ~25% of the forward:
fixed by the lane-contiguous stash layout and vmcnt-counted waits.)
"""
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from scripts.microbench import timeit  # noqa: E402


def run(C, L, prec):
    from masters_thesis_amd.ops.lstm import padded_rows

    dev = "cuda"
    N, T, F, H = 100, 60, 3, 64
    Np = padded_rows(N)
    k = 1 / math.sqrt(H)
    ws = []
    for l in range(L):
        fin = F if l == 0 else H
        for s in ((4 * H, fin), (4 * H, H), (4 * H,), (4 * H,)):
            ws.append((torch.rand(s, device=dev) * 2 - 1) * k)
    x = torch.randn(N, T, F, device=dev)
    E = torch.empty(0, device=dev)
    hseq = [torch.empty((T, Np, H), device=dev) for _ in range(L)]
    stash = [torch.empty(T * Np * 5 * H, device=dev) for _ in range(L)]
    flags = torch.zeros(C.lstm_stack_flag_words(Np), device=dev, dtype=torch.int32)
    seeds = torch.zeros(8, dtype=torch.int64, device=dev)
    gran = torch.zeros(max(L - 1, 1) * T * Np * H, dtype=torch.int64, device=dev)

    def fwd():
        C.lstm_stack_fwd(H, prec, F, x, ws[0::4], ws[1::4], ws[2::4], ws[3::4], hseq, [E] * L, [E] * L, stash, seeds, 0.0,
                         flags, N, Np, T, gran)

    dG = [torch.empty((T, Np, 4 * H), device=dev) for _ in range(L)]
    form = 0  # the dX hand-off: fp32 rows + progress words
    dX = [torch.zeros((T, Np, (2 if form != 0 else 1) * H), device=dev) for _ in range(L - 1)] + [E]
    dh = torch.randn(N, H, device=dev)

    inp = [x] + hseq[:-1]
    grads = [[torch.zeros_like(ws[4 * l + k]) for l in range(L)] for k in range(4)]

    def bwd():
        C.lstm_stack_bwd(H, prec, F, stash, ws[1::4], ws[0::4], dh, dG, dX, hseq, inp, [], [], [], seeds, 0.0, False, flags,
                         N, Np, T, form)

    def bwd_fused():
        C.lstm_stack_bwd(H, prec, F, stash, ws[1::4], ws[0::4], dh, dG, dX, hseq, inp, grads, [], [], seeds, 0.0, False,
                         flags, N, Np, T, form)

    def bwd_wgrad():
        bwd()
        for l in range(L):
            C.lstm_wgrad(prec, dG[l], hseq[l], inp[l] if l else x, l == 0, N, Np, T, H, grads[0][l], grads[1][l],
                         grads[2][l], grads[3][l], None)

    tf, tb = timeit(fwd), timeit(bwd)
    tbf, tbw = timeit(bwd_fused), timeit(bwd_wgrad)
    gx = torch.randn(T, Np, 4 * H, device=dev)

    def old_fwd():
        C.lstm_fwd_layer(H, prec, x, ws[0], ws[2], ws[3], None, stash[0], ws[1], hseq[0], N, Np, T)
        for l in range(1, L):
            C.lstm_fwd_layer(H, prec, None, None, None, None, gx, stash[l], ws[4 * l + 1], hseq[l], N, Np, T)

    to = timeit(old_fwd)
    print(f"L={L} prec={prec}: stack fwd {tf:7.1f} us  bwd {tb:7.1f} us  bwd+fused wgrad {tbf:7.1f} us  "
          f"bwd then {L} wgrad kernels {tbw:7.1f} us | per-layer fwd {to:7.1f} us", flush=True)


def main():
    from masters_thesis_amd.ops import _lib

    C = _lib.lib()
    for L in (1, 2, 4, 8):
        run(C, L, 1)


if __name__ == "__main__":
    main()
