"""One-shot xGMI all-reduce (csrc/allreduce.hip, parallel/xgmi.py) with 2 processes on one MI355X.

The GPU box has one device, so both ranks map each other's fine-grained comm buffers on the SAME GPU
(IPC + peer mapping, gloo process group for the handle exchange): this exercises the whole protocol —
IPC export/import, the parity double buffer, epoch flags, the bounded waits, rank-order summation,
graph capture of the kernel — but not the xGMI link itself (that is the driver's 8-GPU scaling run).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _expected(n, world, rnd):
    out = torch.zeros(n, dtype=torch.float64)
    for r in range(world):
        g = torch.Generator().manual_seed(1000 * rnd + r)
        out += torch.randn(n, generator=g).double()
    return out


def _worker(rank, world, port, n, rounds, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), MTA_ALLREDUCE="xgmi")
    try:
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from masters_thesis_amd.parallel.xgmi import XgmiAllReduce

        dev = torch.device("cuda", 0)
        ar = XgmiAllReduce.create(n, dev)
        assert ar is not None
        worst = 0.0
        for rnd in range(rounds):
            g = torch.Generator().manual_seed(1000 * rnd + rank)
            x = torch.randn(n, generator=g).to(dev)
            ar.allreduce_(x)
            torch.cuda.synchronize()
            worst = max(worst, (x.double().cpu() - _expected(n, world, rnd)).abs().max().item())
        # graph-captured: the epoch lives on the device, replays advance it
        buf = torch.zeros(n, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ar.allreduce_(buf)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        dist.barrier()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            ar.allreduce_(buf)
        for rnd in range(rounds, rounds + 5):
            g = torch.Generator().manual_seed(1000 * rnd + rank)
            buf.copy_(torch.randn(n, generator=g).to(dev))
            graph.replay()
            torch.cuda.synchronize()
            worst = max(worst, (buf.double().cpu() - _expected(n, world, rnd)).abs().max().item())
        ar.check_health()
        ar.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, worst, None))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(240)
@pytest.mark.parametrize("n", [51_200 + 1024, 1 << 20])
def test_xgmi_allreduce_two_processes_one_gpu(n):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 20, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, worst, err in res:
        assert err is None, (rank, err)
        assert worst <= 1e-5, (rank, worst)
