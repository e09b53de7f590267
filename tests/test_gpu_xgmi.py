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
        ar.force_twoshot = twoshot  # None: the size / world based choice
        if twoshot is None:
            assert ar.twoshot(n) == (n * 4 > 512 * 1024 and world > 2)
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


def _overlap_worker(rank, world, port, q):
    """FlatDDP backward-overlapped sync (parallel/ddp.py): layer gradients reported by grad_ready() during a
    simulated backward are reduced on the side stream, the rest at allreduce_grads(); eager and captured + replayed."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), MTA_ALLREDUCE="xgmi")
    try:
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from masters_thesis_amd.ops.optim import FlatParameters
        from masters_thesis_amd.parallel.ddp import FlatDDP, grad_ready

        dev = torch.device("cuda", 0)
        shapes = [(256, 184), (256,), (256,), (256,), (512, 256), (512,), (512,), (512,), (1, 512), (1,)]
        params = [torch.nn.Parameter(torch.zeros(*s, device=dev)) for s in shapes]
        flat = FlatParameters(params)
        ddp = FlatDDP(flat)
        assert ddp.xgmi is not None and ddp.overlap
        ddp.overlap_min_bytes = 4096
        srcs = [torch.zeros(p.numel(), device=dev) for p in params]

        def step():
            ddp.begin_backward()
            for i in (9, 8, 7, 6, 5, 4):  # "top layer first", as a backward produces them
                params[i].grad.view(-1).copy_(srcs[i] * 2.0)
            grad_ready(params[4].grad, params[5].grad)          # overlapped (side stream)
            for i in (3, 2, 1, 0):
                params[i].grad.view(-1).copy_(srcs[i] * 2.0)
            grad_ready(params[0].grad, params[1].grad)          # overlapped
            ddp.allreduce_grads()                                # the rest + join

        def fill(rnd):
            for i, s in enumerate(srcs):
                s.copy_(_data(s.numel(), rank, 100 * rnd + i).to(dev))

        def check(rnd):
            worst = 0.0
            for i, p in enumerate(params):
                exp = 2.0 * sum(_data(srcs[i].numel(), r, 100 * rnd + i).double() for r in range(world))
                worst = max(worst, (p.grad.view(-1).double().cpu() - exp).abs().max().item())
            return worst

        worst = 0.0
        fill(0)
        step()
        torch.cuda.synchronize()
        worst = max(worst, check(0))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            fill(1)
            step()  # warm-up on the capture stream
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                step()
        torch.cuda.synchronize()
        for rnd in (2, 3):
            fill(rnd)
            torch.cuda.synchronize()
            g.replay()
            torch.cuda.synchronize()
            worst = max(worst, check(rnd))
        assert ddp.xgmi.timeouts() == 0
        q.put((rank, worst, None))
        dist.barrier()
        ddp.xgmi.close()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, None, traceback.format_exc()))


def test_overlapped_gradient_sync_two_processes_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_overlap_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, worst, err in res:
        assert err is None, err
        assert worst < 1e-4, (rank, worst)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [4 * 262_147, 4 * 1_000_003])
def test_xgmi_allreduce_four_processes_auto_two_shot_uneven(n):
    """world = 4: the size-based choice (None = auto) picks two-shot for these > 512 KB buckets, and
    n / 4 float4 is odd, so the reduce-scatter chunks are uneven (the last owner gets a short chunk)."""
    world = 4
    assert (n // 4) % world != 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, None, 3, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=280) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    for rank, worst, err in res:
        assert err is None, (rank, err)
        assert worst <= 2e-5, (rank, worst)
