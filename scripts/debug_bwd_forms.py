"""Run-to-run determinism and A/B of the pipelined LSTM forward forms on identical inputs (MTA_LSTM_DEC=0: barrier
forward, 1: decoupled forward; the backward is the barrier body in both): max relative difference of the output and
of each parameter gradient between runs of one form, and between the forms.  Usage: python scripts/debug_bwd_forms.py"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from masters_thesis_amd.ops import lstm as op  # noqa: E402


def run(form, x, ws, R, L, prec):
    os.environ["MTA_LSTM_DEC"] = form
    wg = [w.clone().requires_grad_(True) for w in ws]
    out = op.lstm_last_hidden(x, wg, L, 0.0, True, prec)
    (out * R).sum().backward()
    torch.cuda.synchronize()
    return out.detach().clone(), [w.grad.clone() for w in wg]


def rel(a, b):
    oa, ga = a
    ob, gb = b
    out = ((oa - ob).abs().max() / oa.abs().max().clamp_min(1e-9)).item()
    g = max(((p - q).abs().max() / p.abs().max().clamp_min(1e-9)).item() for p, q in zip(ga, gb))
    return f"out {out:.1e} grad {g:.1e}"


for (N, T, F, H, L) in [(100, 60, 3, 64, 2), (100, 20, 3, 64, 3), (100, 60, 3, 64, 4), (37, 20, 5, 64, 3)]:
    for prec in ["bf16x3", "high", "highest"]:
        torch.manual_seed(1)
        x = torch.randn(N, T, F, device="cuda")
        k = 1.0 / math.sqrt(H)
        ws = []
        for l in range(L):
            fin = F if l == 0 else H
            for shape in ((4 * H, fin), (4 * H, H), (4 * H,), (4 * H,)):
                ws.append(((torch.rand(shape) * 2 - 1) * k).cuda())
        R = torch.randn(N, H, device="cuda")
        r = {f: [run(f, x, ws, R, L, prec) for _ in range(3)] for f in ("0", "1")}
        line = f"N={N} T={T} H={H} L={L} {prec:8s}"
        for f in ("0", "1"):
            line += f" | rerun[{f}] {rel(r[f][0], r[f][1])}, {rel(r[f][0], r[f][2])}"
        line += f" | 1vs0 {rel(r['0'][0], r['1'][0])}"
        print(line, flush=True)
