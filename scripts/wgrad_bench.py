"""LSTM weight-gradient kernel timing sweep (chunking, atomics on/off) on the GPU."""
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from scripts.microbench import timeit  # noqa: E402


def main():
    from masters_thesis_amd.ops import _lib

    C = _lib.lib(required=True)
    dev = "cuda"
    for (N, T, H, F, bf) in ((100, 60, 64, 3, True), (100, 60, 64, 64, False), (800, 60, 64, 64, False)):
        Np = (N + 15) // 16 * 16
        dG = torch.randn(T * Np, 4 * H, device=dev)
        hseq = torch.randn(T, Np, H, device=dev)
        inp = torch.randn(N, T, F, device=dev) if bf else torch.randn(T * Np, F, device=dev)
        g = [torch.zeros(4 * H, F, device=dev), torch.zeros(4 * H, H, device=dev), torch.zeros(4 * H, device=dev),
             torch.zeros(4 * H, device=dev)]
        for prec in (0, 1, 2):
            for tc in ("1", "2", "4"):
                for noat in (False, True):
                    os.environ["MTA_WGRAD_TC"] = tc
                    if noat:
                        os.environ["MTA_WGRAD_NOATOMIC"] = "1"
                    else:
                        os.environ.pop("MTA_WGRAD_NOATOMIC", None)
                    t = timeit(lambda: C.lstm_wgrad(prec, dG, hseq, inp, bf, N, Np, T, H, *g, None))
                    print(f"N={N} F={F} prec={prec} tc={tc} atomics={'off' if noat else 'on '} {t:7.1f} us",
                          flush=True)
    os.environ.pop("MTA_WGRAD_NOATOMIC", None)
    os.environ.pop("MTA_WGRAD_TC", None)


if __name__ == "__main__":
    main()
