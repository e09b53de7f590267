"""Accuracy of the pipelined LSTM per matmul precision against an fp64 CPU reference (headline shape:
N=100 sequences, T=60, F=3, H=64, L=2; B = 1 window).  Prints forward max |err| / max |h| and per-weight gradient
max |err| / max |g| for highest (fp32 MFMA), high (fwd f16x2 + bwd bf16x3), bf16x3, medium (bf16).
    python scripts/lstm_prec_err.py   (GPU)"""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from test_gpu_lstm_pipeline import _ref, _weights  # noqa: E402

from masters_thesis_amd.ops import lstm as op  # noqa: E402


def main():
    N, T, F, H, L = 100, 60, 3, 64, 2
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, T, F, generator=g)
    ws = _weights(F, H, L)
    ref, ws64 = _ref(x, ws, L)
    ref.sum().backward()
    for prec in ("highest", "high", "bf16x3", "medium"):
        wg = [w.cuda().requires_grad_(True) for w in ws]
        out = op.lstm_last_hidden(x.cuda(), wg, L, 0.0, True, prec)
        out.sum().backward()
        torch.cuda.synchronize()
        ferr = (out.double().cpu() - ref.detach()).abs().max().item() / ref.abs().max().item()
        gerr = max((w.grad.double().cpu() - r.grad).abs().max().item() / r.grad.abs().max().item()
                   for w, r in zip(wg, ws64))
        print(f"{prec:8s} forward rel err {ferr:.2e}   worst weight-grad rel err {gerr:.2e}", flush=True)


if __name__ == "__main__":
    main()
