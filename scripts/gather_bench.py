"""Standalone timing of the in-graph batch gather (csrc/lstm_aux.hip gather_batch_kernel) on the LSTM data shapes:
per-call us at B = 1 / 8 / 64 windows (100 stocks x (60 x 3 inputs, 30 x 4 targets), factors, inv_psi), against a
torch index_select of the same rows.  python scripts/gather_bench.py"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from masters_thesis_amd.data.loaders import TensorBatchLoader
    from masters_thesis_amd.ops import _lib

    _lib.lib(required=True)
    dev = "cuda"
    W = 512
    tensors = [torch.randn(W, 100, 60, 3, device=dev), torch.randn(W, 100, 30, 4, device=dev),
               torch.randn(W, 2, device=dev), torch.rand(W, 100, device=dev)]
    for B in (1, 8, 64):
        ld = TensorBatchLoader(tensors, B, shuffle=True, seed=0)
        ld.begin_epoch(0)
        n = min(ld._nfull, 40)
        for _ in range(3):
            ld.gather_static()
        ld.begin_epoch(1)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(n):
            ld.gather_static()
        b.record()
        torch.cuda.synchronize()
        us = a.elapsed_time(b) * 1e3 / n
        idx = torch.randperm(W, device=dev)[:B]
        a.record()
        for _ in range(n):
            for t in tensors:
                t.index_select(0, idx)
        b.record()
        torch.cuda.synchronize()
        us_t = a.elapsed_time(b) * 1e3 / n
        mb = sum(t[0].numel() * 4 for t in tensors) * B / 1e6
        print(f"B={B:3d} {mb:6.2f} MB  gather_batch {us:7.2f} us/call   torch index_select x4 {us_t:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
