"""Local cost of the xGMI all-reduce kernel (csrc/allreduce.hip) with 2 (or 4) processes on ONE MI355X.

Everything but the link itself: the pushes land in this GPU's HBM, so this measures the kernel's own overhead
(flag protocol, fine-grained inbox reads, block count) per bucket size and form.  Prints one JSON line per
(size, form): mean us over the timed calls, algorithm bandwidth = bucket bytes / time.
    python scripts/xgmi_local_bench.py [--world 2] [--iters 50]"""
import argparse
import json
import os
import socket
import sys
from pathlib import Path

import torch
import torch.multiprocessing as mp

REPO = Path(__file__).resolve().parents[1]
SIZES = [51_200 + 1024, 800 * 1024, 13 * 1024 * 1024]  # floats: LSTM small 204 KB, transformer 3.2 MB, mlp_large 52 MB


def _worker(rank, world, port, iters, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), MTA_ALLREDUCE="xgmi")
    sys.path.insert(0, str(REPO))
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from masters_thesis_amd.parallel.xgmi import XgmiAllReduce

    dev = torch.device("cuda", 0)
    ar = XgmiAllReduce.create(max(SIZES), dev)
    out = []
    for n in SIZES:
        x = torch.randn(n, device=dev)
        for two in (False, True):
            ar.force_twoshot = two
            for _ in range(5):
                ar.allreduce_(x)
            torch.cuda.synchronize()
            dist.barrier()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                ar.allreduce_(x)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / iters * 1e3
            out.append({"bytes": n * 4, "form": "two-shot" if two else "one-shot", "us": round(us, 2),
                        "algo_GBps": round(n * 4 / us / 1e3, 1)})
            x.div_(world)  # keep the values bounded
    ar.check_health()
    q.put((rank, out))
    dist.barrier()
    ar.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, a.world, port, a.iters, q)) for r in range(a.world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    knobs = {"world": a.world}
    for i, r0 in enumerate(res[0]):
        worst = max(res[r][i]["us"] for r in res)
        print(json.dumps({**knobs, **r0, "us": worst, "algo_GBps": round(r0["bytes"] / worst / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
