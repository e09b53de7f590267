"""Run-to-run determinism of the pipelined LSTM backward's recurrence: dG / dX of every layer (no fused weight
gradients), 6 reruns against the first.
(r6: this located the decoupled backward's race, profiles/r6_lstm_dec/r6r_bwd_race.txt.)
Usage: python scripts/debug_bwd_race.py [L] [prec]"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from masters_thesis_amd.ops.lstm import lib, padded_rows

    C = lib()
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    prec = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # 1 = bf16x3 (csrc/common.h PREC_*)
    dev = "cuda"
    N, T, F, H = 100, 60, 3, 64
    Np = padded_rows(N)
    torch.manual_seed(0)
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
    C.lstm_stack_fwd(H, prec, F, x, ws[0::4], ws[1::4], ws[2::4], ws[3::4], hseq, [E] * L, [E] * L, stash, seeds,
                     0.0, flags, N, Np, T, gran)
    dh = torch.randn(N, H, device=dev)
    inp = [x] + hseq[:-1]

    def bwd(form):
        dG = [torch.full((T, Np, 4 * H), float("nan"), device=dev) for _ in range(L)]
        dX = [torch.zeros((T, Np, (2 if form else 1) * H), device=dev) for _ in range(L - 1)] + [E]
        C.lstm_stack_bwd(H, prec, F, stash, ws[1::4], ws[0::4], dh, dG, dX, hseq, inp, [], [], [], seeds, 0.0, False,
                         flags, N, Np, T, form)
        torch.cuda.synchronize()
        dX = [d[..., 0::2] if form else d for d in dX[:-1]]  # granules: value bits in the even floats
        return dG, dX

    ref = bwd(0)
    for form in (0,):
        for rep in range(6):
            dG, dX = bwd(form)
            msg = []
            for l in range(L):
                d = (dG[l][:, :N] - ref[0][l][:, :N]).abs()
                sc = ref[0][l][:, :N].abs().max().item()
                bad = (d.amax(dim=(1, 2)) > 1e-5 * sc).nonzero().flatten().tolist()
                msg.append(f"dG[{l}] max {d.max().item() / sc:.1e} steps {bad[:6]}{'...' if len(bad) > 6 else ''}")
            for l in range(L - 1):
                d = (dX[l][:, :N] - ref[1][l][:, :N]).abs()
                sc = ref[1][l][:, :N].abs().max().item()
                msg.append(f"dX[{l}] max {d.max().item() / max(sc, 1e-30):.1e}")
            print(f"L={L} prec={prec} form={form} rep={rep}: " + " | ".join(msg), flush=True)


if __name__ == "__main__":
    main()
