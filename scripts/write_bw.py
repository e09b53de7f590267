"""HBM write-bandwidth yardstick for the GEMM epilogues: 64 MB written by the extension's zero-fill kernel, by
torch fill_, and copied (read + write), timed with events (median of 20)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    from masters_thesis_amd.ops import _lib

    C = _lib.lib(required=True)
    for mb in (16, 64, 256):
        n = mb * (1 << 20) // 4
        x = torch.empty(n, device="cuda")
        y = torch.empty(n, device="cuda")
        for name, fn, nbytes in [("zero_kernel", lambda: C.zero_(x), n * 4), ("torch_fill", lambda: x.fill_(1.0), n * 4),
                                 ("torch_copy", lambda: y.copy_(x), 2 * n * 4)]:
            us = timeit(fn)
            print(json.dumps({"op": name, "MB": mb, "us": round(us, 2), "TB_per_s": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
