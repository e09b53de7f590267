"""Grouped weight-gradient launch (csrc/gemm.hip gemm_group_kernel) on the transformer_encoder B=1 backward's set:
4 layers x {dW2 (128 x 512), dW1 (512 x 128) on k-contiguous images; dWo (128 x 128), dWqkv (384 x 128) on [K][rows]
operands} + the embedding's dWe (128 x 8), K = 6,272 tokens.  Time of the two grouped launches (p50 of 20) and the
worst relative error against fp32 PyTorch.
    python scripts/wgrad_group_bench.py
(The round-5 tile / workgroup-target sweep that set GROUP_WGS: profiles/r5_wgrad_group_sweep.jsonl.)"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])


def run():
    from masters_thesis_amd.ops import _lib
    from masters_thesis_amd.ops import extras as X

    _lib.lib(required=True)
    dev = "cuda"
    torch.manual_seed(0)
    K = 6272
    probs = []
    for _ in range(4):
        for M, N, nn in ((128, 512, True), (512, 128, True), (128, 128, False), (384, 128, False)):
            if nn:
                A = torch.randn(M, K, device=dev).bfloat16()
                B = torch.randn(N, K, device=dev).bfloat16()
            else:
                A = torch.randn(K, M, device=dev).bfloat16()
                B = torch.randn(K, N, device=dev).bfloat16()
            probs.append((nn, A, B, M, N, torch.zeros(M, N, device=dev), torch.zeros(M, device=dev)))
    probs.append((False, torch.randn(K, 128, device=dev).bfloat16(), torch.randn(K, 8, device=dev).bfloat16(), 128, 8,
                  torch.zeros(128, 8, device=dev), torch.zeros(128, device=dev)))

    def step():
        for nn, A, B, M, N, out, bg in probs:
            ks = X.wgrad_split(M, N, K)
            if nn:
                X.gemm(0, A, B, M, N, K, K, K, flags=X.EPI_ACCUM, out_f32=out, ldc=N, n_store=N, ksplit=ks, group=True)
            else:
                X.gemm(2, A, B, M, N, K, M, N, flags=X.EPI_ACCUM, out_f32=out, ldc=N, n_store=N, ksplit=ks,
                       bias_grad=bg, group=True)
        X.gemm_group_flush()

    step()
    torch.cuda.synchronize()
    err = 0.0
    for nn, A, B, M, N, out, bg in probs:
        ref = A.float() @ B.float().t() if nn else A.float().t() @ B.float()
        err = max(err, ((out - ref).abs().max() / ref.abs().max()).item())
    ts = []
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(20):
        a.record()
        step()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    flop = sum(2.0 * M * N * K for _, _, _, M, N, _, _ in probs)
    us = ts[len(ts) // 2]
    print(json.dumps({"us_p50": round(us, 1),
                      "tflops": round(flop / us / 1e6, 1), "rel_err": err}), flush=True)


if __name__ == "__main__":
    run()
