"""Data-parallel correctness without a cluster: 2 gloo ranks on the CPU.

World-size-2 training with one window per rank must follow the same trajectory as a
single process with a global batch of two windows (MSE: mean of per-rank means ==
global mean; the sharded sampler hands rank r the windows idx[r::2]), and the epoch
metrics must be synchronised across ranks.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(W=12):
    g = torch.Generator().manual_seed(0)
    return [torch.randn(W, 100, 20, 3, generator=g), torch.randn(W, 100, 10, 4, generator=g),
            torch.stack([torch.randn(W, generator=g) * 0.1, torch.rand(W, generator=g) + 0.2], -1),
            torch.rand(W, 100, generator=g) * 3 + 1]


def _train(rank, world, batch, steps, out):
    from masters_thesis_amd.data.datamodule import TensorBatchLoader
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import FinancialLstmMse
    from masters_thesis_amd.parallel import dist as pdist

    torch.manual_seed(7 + rank)  # different init per rank: the DDP broadcast must fix it
    model = FinancialLstmMse(hidden_size=16, num_layers=2, dropout=0.0, learning_rate=1e-2)
    ld = TensorBatchLoader(_data(), batch, shuffle=True, seed=0, rank=rank, world_size=world)
    tr = Trainer(gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False, accelerator="cpu")
    tr._setup_env()
    tr._setup_model(model)
    tr._configure_optimizers(model)
    model.train()
    step = tr.make_train_stepper(ld)
    for _ in range(steps):
        step()
    ms = tr._compute_stage_metrics("train")
    torch.save({"params": tr.flat.data.clone(), "mse": float(ms["loss/mse/train"])}, out)
    pdist.destroy()


def _worker(rank, world, port, tmp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from masters_thesis_amd.parallel import dist as pdist

    pdist.init_distributed(backend="gloo", device="cpu")
    _train(rank, world, 1, 5, os.path.join(tmp, f"rank{rank}.pt"))


@pytest.mark.timeout(300)
def test_ddp_two_ranks_equals_single_process_global_batch(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "rank0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "rank1.pt", weights_only=True)
    torch.testing.assert_close(r0["params"], r1["params"], rtol=0, atol=0)  # replicas stay identical
    assert r0["mse"] == r1["mse"]  # synced metric
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    torch.manual_seed(7)
    _train(0, 1, 2, 5, str(tmp_path / "single.pt"))
    s = torch.load(tmp_path / "single.pt", weights_only=True)
    torch.testing.assert_close(r0["params"], s["params"], rtol=1e-5, atol=1e-6)
    assert abs(r0["mse"] - s["mse"]) < 1e-5 * abs(s["mse"])


@pytest.mark.timeout(600)
def test_bench_four_gloo_ranks_whole_path(tmp_path):
    """bench.py under torch.distributed.run with 4 gloo ranks on the CPU: the driver's multi-GPU contract
    (one JSON line from rank 0, whole-job value, n_gpus, weak-scaling global batch, gradient all-reduce) on the
    same code path the MI355X run takes, minus the devices."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    repo = Path(__file__).resolve().parents[1]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), str(repo / "bench.py"), "--gpus", "4", "--steps", "3",
           "--warmup", "1", "--n-samples", "20000"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["steps"] == 3 and rec["warmup"] == 1 and rec["scaling"] == "weak"
    assert rec["config"]["global_batch"] == 4 and rec["config"]["parallelism"] == "dp4"
    assert rec["allreduce"] == "gloo" and rec["value"] > 0


def test_overlapped_sync_reduces_every_range_once():
    """Backward-overlapped gradient sync bookkeeping (parallel/ddp.py + parallel/overlap.py): ranges reported by
    grad_ready() are launched at once when large enough (4-float aligned interior), the rest of the flat gradient
    goes at allreduce_grads(); together every element is reduced exactly once, in a rank-independent order."""
    from masters_thesis_amd.ops.optim import FlatParameters
    from masters_thesis_amd.parallel import overlap
    from masters_thesis_amd.parallel.ddp import FlatDDP, grad_ready

    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.randn(*s)) for s in [(64, 33), (64,), (7,), (128, 64), (128,), (3, 5)]]
    flat = FlatParameters(params)
    ddp = FlatDDP(flat)
    ddp.world = 2  # drive the multi-rank path with a recording reducer instead of a process group
    ddp.overlap_min_bytes = 1024
    calls = []
    ddp._reduce_fn = lambda a, b: calls.append((a, b))
    ddp.begin_backward()
    assert overlap.ACTIVE is ddp
    grad_ready(params[3].grad, params[4].grad)  # 128x64 + 128: launched now
    early = list(calls)
    assert len(early) == 1 and early[0][0] % 4 == 0 and early[0][1] % 4 == 0
    grad_ready(params[2].grad)                  # 7 floats: too small, deferred to the final sync
    assert calls == early
    ddp.allreduce_grads()
    assert overlap.ACTIVE is None
    cover = torch.zeros(flat.padded, dtype=torch.int32)
    for a, b in calls:
        assert a % 4 == 0 and b % 4 == 0
        cover[a:b] += 1
    assert bool((cover == 1).all()), "every element of the flat gradient reduced exactly once"
    # a second step re-arms cleanly
    calls.clear()
    ddp.begin_backward()
    ddp.allreduce_grads()
    assert sum(b - a for a, b in calls) == flat.padded


def test_xgmi_range_channel_invariant():
    """FlatDDP.channel_of: a range keeps its first channel; a range overlapping a different registered range raises
    (csrc/allreduce.hip's parity double buffer is per channel, its inbox slots per flat offset: ADVICE r3)."""
    import pytest
    import torch

    from masters_thesis_amd.ops.optim import FlatParameters
    from masters_thesis_amd.parallel.ddp import FlatDDP

    flat = FlatParameters([torch.nn.Parameter(torch.zeros(4096))])
    ddp = FlatDDP(flat)
    assert ddp.channel_of(0, 1024) == 0
    assert ddp.channel_of(1024, 4096) == 1
    assert ddp.channel_of(0, 1024) == 0 and ddp.channel_of(1024, 4096) == 1
    with pytest.raises(RuntimeError, match="channel invariant"):
        ddp.channel_of(0, 4096)
