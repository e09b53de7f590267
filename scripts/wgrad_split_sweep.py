"""Split-K sweep of the transformer's weight-gradient GEMM shapes (long K = tokens, small fp32 output accumulated with
EPI_ACCUM): time per launch for each ksplit, NN form (operands k-contiguous) and the weight-gradient form (mode 2)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/", 2)[0])
from masters_thesis_amd.ops.extras import EPI_ACCUM, gemm, wgrad_split  # noqa: E402

dev = torch.device("cuda:0")
K = 6240
for M, N in [(128, 512), (512, 128), (384, 128), (128, 128)]:
    for mode in (0, 2):
        if mode == 0:
            A = torch.randn(M, K, device=dev).bfloat16()
            B = torch.randn(N, K, device=dev).bfloat16()
            lda = ldb = K
        else:
            A = torch.randn(K, M, device=dev).bfloat16()
            B = torch.randn(K, N, device=dev).bfloat16()
            lda, ldb = M, N
        out = torch.zeros(M, N, device=dev)
        ref = (A.float() @ B.float().T) if mode == 0 else (A.float().T @ B.float())
        res = []
        for ks in (1, 2, 4, 8, 16, 32, 48):
            out.zero_()
            gemm(mode, A, B, M, N, K, lda, ldb, flags=EPI_ACCUM, out_f32=out, ksplit=ks)
            torch.cuda.synchronize()
            err = ((out - ref).norm() / ref.norm()).item()
            for _ in range(10):
                gemm(mode, A, B, M, N, K, lda, ldb, flags=EPI_ACCUM, out_f32=out, ksplit=ks)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(100):
                gemm(mode, A, B, M, N, K, lda, ldb, flags=EPI_ACCUM, out_f32=out, ksplit=ks)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 10.0
            res.append(f"ks={ks}:{us:.1f}us(err {err:.0e})")
        print(f"M={M} N={N} K={K} mode={mode} default ks={wgrad_split(M, N, K)}: " + " ".join(res), flush=True)
