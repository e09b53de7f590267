"""Split-K A/B of the transformer's weight-gradient GEMMs (dY^T X over M = 6,272 tokens) on the 128-tile path:
time per ksplit for each (out, in) shape.  python scripts/wgrad_split_ab.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.extras import EPI_ACCUM, gemm, gemm_flush

    _lib.lib(required=True)
    K = 6272
    for M, N in ((512, 128), (128, 512), (384, 128), (128, 128)):
        A = torch.randn(K, M, device="cuda").bfloat16()
        B = torch.randn(K, N, device="cuda").bfloat16()
        out = torch.zeros(M, N, device="cuda")
        res = []
        for ks in (1, 2, 4, 8, 16, 32, 48):
            def fn():
                gemm(2, A, B, M, N, K, M, N, flags=EPI_ACCUM, out_f32=out, ldc=N, n_store=N, ksplit=ks)
                gemm_flush()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(20):
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            res.append(f"ks={ks}: {ts[10]:.1f} us")
        print(f"wgrad {M}x{N}x{K}: " + ", ".join(res), flush=True)


if __name__ == "__main__":
    main()
