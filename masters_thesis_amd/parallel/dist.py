"""Process-group bootstrap: one process per GPU, RCCL over xGMI.

The reference gets DDP implicitly from Lightning (`train.py:169-180`).  Here the
launcher contract is explicit: ``torchrun``/``torch.distributed.run`` (or the
``gpu_pool`` launcher) sets ``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_*``;
``init_distributed()`` binds the process to ``cuda:LOCAL_RANK`` *before* creating
the ``"nccl"`` (= RCCL on ROCm) group, and falls back to ``gloo`` on CPU-only hosts
(multi-process CPU tests).  Collective timeouts surface as exceptions (failure
detection) instead of silent hangs.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    device: torch.device = torch.device("cpu")
    backend: Optional[str] = None

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_global_zero(self) -> bool:
        return self.rank == 0


_ENV: Optional[DistEnv] = None


def env_world_size() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0, device: Optional[str] = None) -> DistEnv:
    """Initialise (once) from torchrun-style env vars; returns the rank/device description."""
    global _ENV
    if _ENV is not None:
        return _ENV
    world = env_world_size()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = device != "cpu" and torch.cuda.is_available()
    if use_gpu:
        # ranks beyond the visible devices share them (gloo rehearsal of N ranks on a 1-GPU box)
        idx = local_rank % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
    else:
        dev = torch.device("cpu")
    be = None
    if world > 1:
        # RCCL needs one GPU per rank: ranks sharing a GPU (a rehearsal on fewer GPUs than ranks) take gloo for the
        # host collectives; their gradient sync is still the xGMI/IPC kernel (parallel/ddp.py)
        shared = use_gpu and int(os.environ.get("LOCAL_WORLD_SIZE", world)) > torch.cuda.device_count()
        be = backend or os.environ.get("MTA_DIST_BACKEND") or ("nccl" if use_gpu and not shared else "gloo")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if not dist.is_initialized():
            kw = {}
            if be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(be, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    _ENV = DistEnv(rank, local_rank, world, dev, be)
    return _ENV


def get_env() -> DistEnv:
    return _ENV if _ENV is not None else DistEnv(device=torch.device("cuda", 0) if torch.cuda.is_available()
                                                 else torch.device("cpu"))


def barrier() -> None:
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_max(x: float, device: torch.device) -> float:
    if not (dist.is_available() and dist.is_initialized()):
        return float(x)
    t = torch.tensor([float(x)], device=device if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_object(obj, src: int = 0):
    if not (dist.is_available() and dist.is_initialized()):
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src)
    return lst[0]


def destroy() -> None:
    global _ENV
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    _ENV = None
