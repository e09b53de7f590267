"""Diagnostics for the pipelined LSTM stack kernel: per-layer, per-timestep error vs fp64."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.lstm import padded_rows

    C = _lib.lib()
    torch.manual_seed(1)
    import os
    cases = [(0, 64, 2, "all"), (0, 64, 2, "zero_wih1"), (0, 64, 2, "zero_whh1"), (0, 64, 2, "zero_bias1"),
             (1, 64, 2, "zero_whh1")]
    for prec, H, L, mode in cases:
        N, T, F = 100, 12, 3
        Np = padded_rows(N)
        x = torch.randn(N, T, F)
        g = torch.Generator().manual_seed(0)
        k = 1 / math.sqrt(H)
        ws = []
        for l in range(L):
            fin = F if l == 0 else H
            for s in ((4 * H, fin), (4 * H, H), (4 * H,), (4 * H,)):
                ws.append((torch.rand(s, generator=g) * 2 - 1) * k)
        if mode == "zero_wih1":
            ws[4].zero_()
        elif mode == "zero_whh1":
            ws[5].zero_()
        elif mode == "zero_bias1":
            ws[6].zero_()
            ws[7].zero_()
        # reference per layer
        inp = x.double()
        refs = []
        for l in range(L):
            h0 = torch.zeros(1, N, H, dtype=torch.float64)
            out, _, _ = torch._VF.lstm(inp, (h0, h0), [w.double() for w in ws[4 * l:4 * l + 4]], True, 1, 0.0, False,
                                       False, True)
            refs.append(out)
            inp = out
        wd = [w.cuda() for w in ws]
        E = torch.empty(0, device="cuda")
        hseq = [torch.full((T, Np, H), float("nan"), device="cuda") for _ in range(L)]
        flags = torch.zeros(C.lstm_stack_flag_words(Np), device="cuda", dtype=torch.int32)
        seeds = torch.zeros(8, dtype=torch.int64, device="cuda")
        gran = torch.zeros(max(L - 1, 1) * T * Np * H, dtype=torch.int64, device="cuda")
        C.lstm_stack_fwd(H, prec, F, x.cuda(), wd[0::4], wd[1::4], wd[2::4], wd[3::4], hseq, [E] * L, [E] * L, [E] * L,
                         seeds, 0.0, flags, N, Np, T, gran)
        torch.cuda.synchronize()
        fl = flags.cpu()
        print(f"[{mode}] prec={prec} H={H} L={L} flags={fl[:256:32].tolist()} ... timeout={fl[-160].item()}", flush=True)
        for l in range(L):
            got = hseq[l].cpu()[:, :N].permute(1, 0, 2).double()
            err = (got - refs[l]).abs().amax(dim=(0, 2))
            print(f"  layer {l}: max err per t = {[round(float(e), 6) for e in err]}", flush=True)


if __name__ == "__main__":
    main()
