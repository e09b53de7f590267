"""bf16 MFMA GEMM (csrc/gemm.hip) micro-benchmark on the extras encoders' shapes: TFLOP/s per mode and the max
error against an fp32 PyTorch reference of the same product.

  python scripts/gemm_bench.py [--json out.jsonl]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

# (name, mode, M, N, K): mode 0 = X W^T, 1 = dY W, 2 = dY^T X (split-K into fp32)
SHAPES = [
    ("mlp_large fwd", 0, 6400, 2048, 2048),
    ("mlp_large dgrad", 1, 6400, 2048, 2048),
    ("mlp_large wgrad", 2, 2048, 2048, 6400),
    ("mlp_large fwd0", 0, 6400, 2048, 184),
    ("tr qkv", 0, 6272, 384, 128),
    ("tr ffn up", 0, 6272, 512, 128),
    ("tr ffn down", 0, 6272, 128, 512),
    ("tr proj", 0, 6272, 128, 128),
    ("tr wgrad ffn", 2, 512, 128, 6272),
    ("sq 4096", 0, 4096, 4096, 4096),
]


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--ab", action="store_true", help="every shape on the default path (-1), the 256x256 kernel forced (1) and the 128-tile path (0)")
    ap.add_argument("--only", default=None, help="substring filter on the shape names")
    ap.add_argument("--variants", default=None, help="comma-separated gemm_set_big values (default: -1, or -1,1,0 with --ab)")
    ap.add_argument("--no-blas", action="store_true")
    args = ap.parse_args()
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops.extras import EPI_ACCUM, gemm, gemm_flush, wgrad_split

    _lib.lib(required=True)
    dev = "cuda"
    torch.manual_seed(0)
    rows = []
    variants = (-1, 1, 0) if args.ab else (-1,)
    if args.variants:
        variants = tuple(int(v) for v in args.variants.split(","))
    shapes = [sh for sh in SHAPES if args.only is None or args.only in sh[0]]
    for (name, mode, M, N, K), big in [(sh, v) for sh in shapes for v in variants]:
        _lib.lib().gemm_set_big(big)
        if mode == 0:
            A = torch.randn(M, K, device=dev).bfloat16()
            B = torch.randn(N, K, device=dev).bfloat16()
            ref = A.float() @ B.float().t()
            out = torch.empty(M, N, device=dev)
            fn = lambda: gemm(0, A, B, M, N, K, K, K, out_f32=out)  # noqa: E731
            ks = 1
        elif mode == 1:
            A = torch.randn(M, K, device=dev).bfloat16()      # dY [M][K=Dout]
            B = torch.randn(K, N, device=dev).bfloat16()      # W [Dout=K][Din=N]
            ref = A.float() @ B.float()
            out = torch.empty(M, N, device=dev)
            fn = lambda: gemm(1, A, B, M, N, K, K, N, out_f32=out)  # noqa: E731
            ks = 1
        else:
            A = torch.randn(K, M, device=dev).bfloat16()      # dY [tokens][M]
            B = torch.randn(K, N, device=dev).bfloat16()      # X [tokens][N]
            ref = A.float().t() @ B.float()
            out = torch.zeros(M, N, device=dev)
            ks = wgrad_split(M, N, K)

            def fn():
                gemm(2, A, B, M, N, K, M, N, flags=EPI_ACCUM, out_f32=out, ldc=N, n_store=N, ksplit=ks)
                gemm_flush()
        out.zero_()
        fn()
        torch.cuda.synchronize()
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        us = timeit(fn)
        tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
        # the vendor library on the same product (torch.matmul -> hipBLASLt, bf16 out, no fused epilogue)
        Ab = A if mode != 2 else A.t()
        Bb = B.t() if mode == 0 else B
        blas_us = float("nan") if args.no_blas else timeit(lambda: torch.matmul(Ab, Bb))
        row = {"shape": name, "big": big, "mode": mode, "M": M, "N": N, "K": K, "ksplit": ks, "us": round(us, 2),
               "tflops": round(tf, 1), "blas_us": round(blas_us, 2),
               "blas_tflops": round(2.0 * M * N * K / (blas_us * 1e-6) / 1e12, 1), "rel_err": err}
        rows.append(row)
        print(json.dumps(row), flush=True)
        assert err < 2e-2, row
    if args.json:
        with open(args.json, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
