"""Fused weight-gradient workgroups of the backward stack kernel vs the standalone wgrad kernel."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.lstm import padded_rows

    C = _lib.lib()
    dev = "cuda"
    torch.manual_seed(0)
    for (L, T, N, F) in ((2, 60, 100, 3), (3, 24, 50, 3), (2, 7, 20, 5)):
        H = 64
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
        C.lstm_stack_fwd(H, 1, F, x, ws[0::4], ws[1::4], ws[2::4], ws[3::4], hseq, [E] * L, [E] * L, stash, seeds, 0.0,
                         flags, N, Np, T)
        dG = [torch.empty((T, Np, 4 * H), device=dev) for _ in range(L)]
        dX = [torch.empty((T, Np, H), device=dev) for _ in range(L - 1)] + [E]
        dh = torch.randn(N, H, device=dev)
        inp = [x] + hseq[:-1]
        ref = [[torch.zeros_like(ws[4 * l + kk]) for l in range(L)] for kk in range(4)]
        C.lstm_stack_bwd(H, 1, F, stash, ws[1::4], ws[0::4], dh, dG, dX, hseq, inp, [], [], [], seeds, 0.0, False, flags,
                         N, Np, T)
        for l in range(L):
            C.lstm_wgrad(1, dG[l], hseq[l], inp[l], l == 0, N, Np, T, H, ref[0][l], ref[1][l], ref[2][l], ref[3][l], None)
        dG_ref = [d.clone() for d in dG]
        for rep in range(3):
            got = [[torch.zeros_like(ws[4 * l + kk]) for l in range(L)] for kk in range(4)]
            C.lstm_stack_bwd(H, 1, F, stash, ws[1::4], ws[0::4], dh, dG, dX, hseq, inp, got, [], [], seeds, 0.0, False,
                             flags, N, Np, T)
            torch.cuda.synchronize()
            errs = []
            for kk in range(4):
                for l in range(L):
                    r, g = ref[kk][l], got[kk][l]
                    errs.append(round(((g - r).abs().max() / r.abs().max().clamp_min(1e-9)).item(), 7))
            dgerr = max((a - b).abs().max().item() for a, b in zip(dG, dG_ref))
            print(f"L={L} T={T} N={N} F={F} rep={rep}: rel err per grad {errs} dG diff {dgerr:.3g} "
                  f"timeout={flags[-160].item()}", flush=True)


if __name__ == "__main__":
    main()
