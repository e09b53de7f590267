"""(Historical: the projection mode it A/Bs was removed after this measurement, profiles/r2_proj_ab.txt.)
A/B timing of the pipelined LSTM forward/backward: projection workgroups (MTA_LSTM_PROJ=1) vs in-workgroup input
waves (0), per (L, dropout), N=100 T=60 H=64 (the headline shape)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from masters_thesis_amd.ops import lstm as op  # noqa: E402


def weights(F, H, L):
    ws = []
    for l in range(L):
        fin = F if l == 0 else H
        for shape in ((4 * H, fin), (4 * H, H), (4 * H,), (4 * H,)):
            ws.append((torch.rand(shape, device="cuda") * 2 - 1) * 0.125)
    return ws


def bench(L, p, proj, reps=200):
    os.environ["MTA_LSTM_PROJ"] = proj
    x = torch.randn(100, 60, 3, device="cuda")
    ws = weights(3, 64, L)
    seeds = torch.zeros(8, dtype=torch.int64, device="cuda")
    for _ in range(10):
        h, st = op.pipelined_forward(x, seeds, 1, p, True, True, ws)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        h, st = op.pipelined_forward(x, seeds, 1, p, True, True, ws)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


for L in (1, 2, 4, 8):
    for p in (0.0, 0.2):
        if L == 1 and p > 0:
            continue
        a = bench(L, p, "1")
        b = bench(L, p, "0")
        print(f"L={L} p={p}: fwd proj {a:.1f} us  legacy {b:.1f} us", flush=True)
op.check_pipeline_health()
