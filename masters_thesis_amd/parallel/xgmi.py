"""One-shot all-reduce over xGMI peer memory (``csrc/allreduce.hip``) for the flat gradient bucket.

Reference: Lightning's implicit DDP all-reduces the gradients with NCCL every step (`train.py:169-180`,
SURVEY §2.6 M2).  On one MI355X node the ranks are fully connected by xGMI (7 point-to-point links per GPU),
so for this workload's small buckets (204 KB for ``model=small``) a ring all-reduce is latency-bound:
2 (N-1) dependent hops.  Here every rank pushes its gradient into a slot of every peer's comm buffer in ONE
kernel (all 7 links at once), signals, and sums the N slots locally in rank order — one launch, no host
involvement, capturable inside the step's HIP graph.

Setup (``XgmiAllReduce.create``): each rank allocates a fine-grained (cross-device coherent) comm buffer,
exports it with ``hipIpcGetMemHandle``, the handles are all-gathered over the process group and every rank
maps every peer's buffer (``hipIpcOpenMemHandle``, lazy peer access).  Before the object is used a
self-check compares it against the process group's own all-reduce on random data for a few rounds; any
mismatch, exception or timeout disables it (``FlatDDP`` then keeps RCCL) and says why.  The kernel bounds
every wait and counts give-ups in a device word that ``check_health`` turns into an exception.

Selection (``MTA_ALLREDUCE``): ``auto`` (default: xGMI when all ranks share one node, the bucket is at most
``max_mb`` and the self-check passes), ``xgmi`` (required: raise if unavailable), ``rccl``.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops._lib import lib

_LIVE: List["XgmiAllReduce"] = []


class XgmiAllReduce:
    def __init__(self, numel: int, device: torch.device, group=None):
        C = lib()
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.numel = int(numel)
        self.cap = -(-self.numel // 4) * 4
        self.device = device
        self._C = C
        self.bytes = C.xgmi_buffer_bytes(self.world, self.cap)
        self.own = C.xgmi_alloc(self.bytes)
        handle = C.xgmi_ipc_handle(self.own)
        handles = [None] * self.world
        dist.all_gather_object(handles, handle.tolist(), group=group)
        self.bufs: List[int] = []
        self._opened: List[int] = []
        for p, h in enumerate(handles):
            if p == self.rank:
                self.bufs.append(self.own)
            else:
                ptr = C.xgmi_ipc_open(torch.tensor(h, dtype=torch.uint8))
                self.bufs.append(ptr)
                self._opened.append(ptr)
        self.ctl = torch.zeros(C.xgmi_ctl_words(), dtype=torch.int32, device=device)
        dist.barrier(group=group)  # every peer mapped every buffer before the first push
        _LIVE.append(self)

    # ------------------------------------------------------------------ use
    def allreduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the ranks of a contiguous fp32 CUDA tensor of at most ``numel`` elements."""
        if t.numel() % 4:
            raise ValueError("xgmi all-reduce needs a multiple of 4 elements")
        self._C.xgmi_allreduce(t, self.cap, self.bufs, self.rank, self.ctl)
        return t

    def timeouts(self) -> int:
        return int(self.ctl[64].item())

    def check_health(self) -> None:
        n = self.timeouts()
        if n:
            self.ctl[64].zero_()
            raise RuntimeError(f"xGMI all-reduce: {n} wait(s) on a peer gave up (that step's gradients are invalid)")

    def close(self) -> None:
        if self in _LIVE:
            _LIVE.remove(self)
        try:
            torch.cuda.synchronize(self.device)
            for p in self._opened:
                self._C.xgmi_ipc_close(p)
            self._C.xgmi_free(self.own)
        except Exception:  # pragma: no cover - teardown at interpreter exit
            pass
        self._opened = []

    # ------------------------------------------------------------------ construction + self-check
    @classmethod
    def create(cls, numel: int, device: torch.device, group=None,
               max_mb: float = float(os.environ.get("MTA_XGMI_MAX_MB", "4"))) -> Optional["XgmiAllReduce"]:
        # one-shot pushes the whole bucket over every link (N-1 copies out per rank): latency-optimal for the LSTM
        # (204 KB) and transformer (3.2 MB) buckets; above a few MB RCCL's ring / two-shot moves ~2x less per link
        # (mlp_large's 52 MB bucket: ~1 ms one-shot vs ~0.25 ms ring at ~50 GB/s per xGMI link)
        """The xGMI all-reduce for this group, or None (with the reason printed once on rank 0) when the
        configuration does not allow it or its self-check against the group's all-reduce fails."""
        mode = os.environ.get("MTA_ALLREDUCE", "auto").lower()
        if mode == "rccl":
            return None
        required = mode == "xgmi"

        def no(reason: str):
            if required:
                raise RuntimeError(f"MTA_ALLREDUCE=xgmi but the xGMI all-reduce is unavailable: {reason}")
            if dist.get_rank(group) == 0:
                print(f"[ddp] xGMI all-reduce off ({reason}); using the process group's all-reduce", flush=True)
            return None

        if not (dist.is_available() and dist.is_initialized()) or device.type != "cuda":
            return no("not a GPU process group")
        world = dist.get_world_size(group)
        local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if world < 2 or world > 8 or local != world:
            return no(f"needs 2..8 ranks on one node (world={world}, local={local})")
        if numel * 4 > max_mb * (1 << 20):
            return no(f"bucket {numel * 4 / 2 ** 20:.1f} MB > {max_mb} MB (ring bandwidth wins)")
        try:
            ar = cls(numel, device, group)
        except Exception as e:  # allocation / IPC unavailable on this platform
            return no(f"setup failed: {e}")
        ok, why = ar._self_check(group)
        ok_all = torch.tensor([1 if ok else 0], device=device, dtype=torch.int32)
        dist.all_reduce(ok_all, op=dist.ReduceOp.MIN, group=group)
        if int(ok_all.item()) != 1:
            ar.close()
            return no(f"self-check failed: {why or 'on another rank'}")
        return ar

    def _self_check(self, group, rounds: int = 6):
        g = torch.Generator(device=self.device).manual_seed(1234 + self.rank)
        n = min(self.cap, 1 << 20)
        try:
            for r in range(rounds):
                x = torch.randn(n, device=self.device, generator=g)
                ref = x.clone()
                dist.all_reduce(ref, group=group)
                self.allreduce_(x)
                torch.cuda.synchronize(self.device)
                if self.timeouts():
                    return False, "peer wait timed out"
                if not torch.allclose(x, ref, rtol=1e-5, atol=1e-5):
                    return False, f"round {r}: max err {(x - ref).abs().max().item():.3g}"
            return True, ""
        except Exception as e:  # pragma: no cover - surfaced through the MIN all-reduce
            return False, str(e)


def check_all_health() -> None:
    for ar in list(_LIVE):
        ar.check_health()
