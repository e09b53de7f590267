"""Timing of the pipelined LSTM stack kernels vs the per-layer kernels (fwd / bwd, L = 1..8).

plain=1 rows use plain (not write-through) hand-off stores, plain=2 also drop the stash / dG stores,
plain=3 also the backward's stash loads: timing probes of the memory-traffic cost only (invalid results).
"""
import math
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from scripts.microbench import timeit  # noqa: E402


def run(C, L, prec, plain):
    from masters_thesis_amd.ops.lstm import padded_rows

    if plain:
        os.environ["MTA_STACK_PLAIN_STORES"] = str(int(plain))
    else:
        os.environ.pop("MTA_STACK_PLAIN_STORES", None)
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
    flags = torch.empty(C.lstm_stack_flag_words(Np), device=dev, dtype=torch.int32)
    seeds = torch.zeros(8, dtype=torch.int64, device=dev)

    def fwd():
        C.lstm_stack_fwd(H, prec, F, x, ws[0::4], ws[1::4], ws[2::4], ws[3::4], hseq, [E] * L, stash, seeds, 0.0,
                         flags, N, Np, T)

    dG = [torch.empty((T, Np, 4 * H), device=dev) for _ in range(L)]
    dX = [torch.empty((T, Np, H), device=dev) for _ in range(L - 1)] + [E]
    dh = torch.randn(N, H, device=dev)

    def bwd():
        C.lstm_stack_bwd(H, prec, stash, ws[1::4], ws[0::4], dh, dG, dX, seeds, 0.0, False, flags, N, Np, T)

    tf, tb = timeit(fwd), timeit(bwd)
    gx = torch.randn(T, Np, 4 * H, device=dev)

    def old_fwd():
        C.lstm_fwd_layer(H, prec, x, ws[0], ws[2], ws[3], None, stash[0], ws[1], hseq[0], N, Np, T)
        for l in range(1, L):
            C.lstm_fwd_layer(H, prec, None, None, None, None, gx, stash[l], ws[4 * l + 1], hseq[l], N, Np, T)

    to = timeit(old_fwd)
    print(f"L={L} plain={int(plain)} prec={prec}: stack fwd {tf:7.1f} us  bwd {tb:7.1f} us | per-layer fwd {to:7.1f} us",
          flush=True)


def main():
    from masters_thesis_amd.ops import _lib

    C = _lib.lib()
    for L in (1, 2, 4, 8):
        for plain in (0, 1, 2, 3):
            run(C, L, 1, plain)
    os.environ.pop("MTA_STACK_PLAIN_STORES", None)


if __name__ == "__main__":
    main()
