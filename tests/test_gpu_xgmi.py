"""xGMI all-reduce (csrc/allreduce.hip, parallel/xgmi.py) with 2 processes on one MI355X.

The GPU box has one device, so both ranks map each other's fine-grained comm buffers on the SAME GPU
(IPC + peer mapping, gloo process group for the handle exchange): this exercises the whole protocol --
collective set-up, IPC export/import, the parity double buffer, per-bucket channels, epoch flags, the bounded
waits, one-shot AND two-shot (reduce-scatter + all-gather), rank-order summation, graph capture and replay --
against an fp64 sum, for buckets of 4 KB to 64 MB, but not the xGMI link itself (that is the driver's 8-GPU
scaling run).
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


def _data(n, rank, rnd):
    g = torch.Generator().manual_seed(1000 * rnd + rank)
    return torch.randn(n, generator=g)


def _expected(n, world, rnd):
    out = torch.zeros(n, dtype=torch.float64)
    for r in range(world):
        out += _data(n, r, rnd).double()
    return out


def _worker(rank, world, port, n, twoshot, rounds, q):
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
        ar.force_twoshot = twoshot
        worst = 0.0
        for rnd in range(rounds):
            x = _data(n, rank, rnd).to(dev)
            ar.allreduce_(x)
            torch.cuda.synchronize()
            worst = max(worst, (x.double().cpu() - _expected(n, world, rnd)).abs().max().item())
        # two buckets on two channels (offsets into the flat buffer), then the same inside a captured graph: the
        # per-channel epochs live on the device, replays advance them
        half = (n // 2) // 4 * 4
        buf = torch.zeros(n, device=dev)

        def two_buckets():
            ar.allreduce_(buf[:half], off=0, channel=0)
            ar.allreduce_(buf[half:], off=half, channel=1)

        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            two_buckets()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        dist.barrier()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            two_buckets()
        for rnd in range(rounds, rounds + 3):
            buf.copy_(_data(n, rank, rnd).to(dev))
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


@pytest.mark.timeout(300)
@pytest.mark.parametrize("twoshot", [False, True])
@pytest.mark.parametrize("n,rounds", [(1024, 6), (51_200 + 1024, 6), (1 << 20, 4), (1 << 24, 2)])
def test_xgmi_allreduce_two_processes_one_gpu(n, rounds, twoshot):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, twoshot, rounds, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=280) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, worst, err in res:
        assert err is None, (rank, err)
        assert worst <= 1e-5 * (1 + (n >= 1 << 24)), (rank, worst)
