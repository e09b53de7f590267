"""Fused clip + Adam(W) launch at the mlp_large size (13.4 M parameters): time per launch and effective HBM rate
(28 B per parameter: p, g, m, v read; p, m, v written), with and without producer-covered gradient ranges.
    python scripts/adam_bench.py [n_params]"""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from masters_thesis_amd.ops._lib import lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 13_393_920
    n -= n % 4
    C = lib(required=True)
    dev = torch.device("cuda", 0)
    p, g, m, v = (torch.randn(n, device=dev) * 1e-2 for _ in range(4))
    v.abs_()
    parts = torch.zeros(C.adam_fused_partials(), device=dev)
    ticket = torch.zeros(1, dtype=torch.int64, device=dev)
    lr = torch.full((1,), 1e-4, device=dev)
    step = torch.zeros(1, device=dev)
    norm = torch.zeros(1, device=dev)
    health = torch.zeros(2, device=dev)
    ext = torch.zeros(8 * 4096, device=dev)
    for mode in ("plain", "covered"):
        cov = ([0], [n // 4 - 1024]) if mode == "covered" else ([], [])
        run = lambda: C.adam_fused(p, g, m, v, parts, ticket, lr, step, 0.9, 0.999, 1e-8, 1e-5, 5.0, 1.0,  # noqa
                                   True, True, norm, health, cov[0], cov[1], ext if cov[0] else None)
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        times = []
        for _ in range(20):
            t0.record()
            run()
            t1.record()
            t1.synchronize()
            times.append(t0.elapsed_time(t1) * 1e3)
        times.sort()
        us = times[len(times) // 2]
        print(json.dumps({"mode": mode, "n": n, "us_p50": round(us, 2), "tb_s": round(28 * n / us / 1e6, 2),
                          "health": health.tolist()}))


if __name__ == "__main__":
    main()
