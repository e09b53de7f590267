"""Per-op latency micro-benchmarks on the GPU (CUDA-event timed, median of repeats)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def timeit(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.lstm import lstm_last_hidden
    import math

    _lib.lib(required=True)
    dev = "cuda"
    H, F, T = 64, 3, 60
    for L in (2, 8):
        for B in (1, 8, 32):
            N = 100 * B
            k = 1 / math.sqrt(H)
            ws = []
            for l in range(L):
                fin = F if l == 0 else H
                for s in ((4 * H, fin), (4 * H, H), (4 * H,), (4 * H,)):
                    ws.append(((torch.rand(s, device=dev) * 2 - 1) * k).requires_grad_(True))
            x = torch.randn(N, T, F, device=dev)
            for prec in ("highest", "high", "medium"):
                def fwd():
                    with torch.no_grad():
                        lstm_last_hidden(x, ws, L, 0.0, False, prec)

                def fwdbwd():
                    out = lstm_last_hidden(x, ws, L, 0.2, True, prec)
                    out.sum().backward()

                tf = timeit(fwd)
                tfb = timeit(fwdbwd)
                print(f"L={L} B={B:3d} N={N:5d} prec={prec:8s} fwd(no-grad) {tf:8.1f} us  fwd+bwd {tfb:8.1f} us",
                      flush=True)
    # torch reference path (MIOpen LSTM) for comparison
    for L in (2,):
        for B in (1, 32):
            N = 100 * B
            lstm = torch.nn.LSTM(F, H, L, batch_first=True, dropout=0.2).to(dev)
            x = torch.randn(N, T, F, device=dev)

            def ref():
                out, _ = lstm(x)
                out[:, -1].sum().backward()

            print(f"[torch nn.LSTM/MIOpen] L={L} B={B} fwd+bwd {timeit(ref):8.1f} us", flush=True)


if __name__ == "__main__":
    main()
