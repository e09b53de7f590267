"""Streaming data path (``datamodule.residency=stream``): pinned host ring + side-stream H2D.

The split stays in page-locked host memory.  ``csrc/host/prefetch.cpp`` worker threads gather
the rows of the next ``slots`` batches into a pinned staging ring (the reference's
``DataLoader(num_workers=4, pin_memory=True)``, `src/data.py:236-238`, without worker processes
or pickling).  Per step the loader issues one ``hipMemcpyAsync`` per tensor on its own copy
stream into the matching slot of a device ring, and the captured step graph gathers the batch
from ring slot ``s mod slots`` with the same device-cursor kernel as the HBM-resident path —
so the graph is identical for both residencies and the copy of batch s+1 overlaps the compute
of batch s.  Events order the ring both ways: a copy into slot k waits until the step that last
read slot k has finished; the step waits until its copy has landed.
"""
from __future__ import annotations

from typing import Iterator, List, Optional

import torch
from torch import Tensor

from ..ops import _lib
from .loaders import TensorBatchLoader


class StreamingLoader:
    def __init__(self, base: TensorBatchLoader, device, slots: int = 3, threads: int = 2,
                 wait_timeout_ms: int = 60_000):
        self.base = base
        self.device = torch.device(device)
        self.batch_size = base.batch_size
        self.slots = max(2, int(slots))
        self.threads = max(1, int(threads))
        self.wait_timeout_ms = int(wait_timeout_ms)
        self.bytes_copied = 0
        self._epoch_idx: Optional[Tensor] = None
        self._pf = None
        self._nfull = 0
        self._s = 0
        if self.device.type == "cuda":
            if any(t.is_cuda for t in base.tensors):
                raise ValueError("StreamingLoader streams from host tensors; got device tensors")
            self._setup_device()

    # ------------------------------------------------------------------ plumbing
    def _setup_device(self) -> None:
        C = _lib.lib(required=True)
        B, R, dev = self.batch_size, self.slots, self.device
        self.host = [t if t.is_pinned() else t.pin_memory() for t in self.base.tensors]
        self.staging = [torch.empty((R * B, *t.shape[1:]), dtype=t.dtype).pin_memory() for t in self.host]
        self.ring = [torch.empty((R * B, *t.shape[1:]), dtype=t.dtype, device=dev) for t in self.host]
        self.static = [torch.empty((B, *t.shape[1:]), dtype=t.dtype, device=dev) for t in self.host]
        max_batches = max(1, len(self.base))
        # perm[s*B + b] = (s mod R)*B + b: the gather kernel reads ring slot s mod R at step s
        s = torch.arange(max_batches).repeat_interleave(B)
        b = torch.arange(B).repeat(max_batches)
        self._perm = ((s % R) * B + b).to(torch.int32).to(dev)
        self._cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self._arrive = torch.zeros(65 * 32, dtype=torch.int32, device=dev)  # gather arrival counters, one line each
        self.copy_stream = torch.cuda.Stream(device=dev)
        self._copied = [torch.cuda.Event() for _ in range(R)]
        self._consumed = [torch.cuda.Event() for _ in range(R)]
        self._consumed_valid = [False] * R
        self._pending: Optional[int] = None  # batch whose staging slot awaits release
        self._pf = C.HostPrefetcher(self.host, self.staging, B, R, self.threads)
        self._row_bytes = sum(t[0].numel() * t.element_size() for t in self.host)

    def supports_static(self) -> bool:
        return self._pf is not None

    def set_epoch(self, epoch: int) -> None:
        self.base.set_epoch(epoch)

    def __len__(self) -> int:
        return len(self.base)

    def __iter__(self) -> Iterator[List[Tensor]]:
        for batch in self.base:
            yield [t.to(self.device, non_blocking=True) for t in batch] if self.device.type == "cuda" else batch

    # ------------------------------------------------------------------ static protocol
    def begin_epoch(self, epoch: int) -> int:
        self.copy_stream.synchronize()  # staging slots of the previous epoch are no longer read
        self.base.set_epoch(epoch)
        idx = self.base.epoch_indices()
        self._epoch_idx = idx
        B = self.batch_size
        self._nfull = idx.numel() // B
        self._pf.start(idx[: self._nfull * B].contiguous(), self._nfull)
        self._cursor.zero_()
        self._arrive.zero_()
        self._s = 0
        self._pending = None
        return self._nfull

    def before_static_step(self) -> None:
        s, B, R = self._s, self.batch_size, self.slots
        if s >= self._nfull:
            raise RuntimeError("StreamingLoader: more static steps than full batches in this epoch")
        slot = self._pf.wait(s, self.wait_timeout_ms)
        if slot < 0:
            raise RuntimeError(f"StreamingLoader: batch {s} not staged (prefetcher {'timeout' if slot == -2 else 'stopped'})")
        rows = slice(slot * B, (slot + 1) * B)
        with torch.cuda.stream(self.copy_stream):
            if self._consumed_valid[slot]:
                self.copy_stream.wait_event(self._consumed[slot])
            for d, h in zip(self.ring, self.staging):
                d[rows].copy_(h[rows], non_blocking=True)
            self._copied[slot].record(self.copy_stream)
        torch.cuda.current_stream().wait_event(self._copied[slot])
        # the previous batch's copy has been queued long enough: free its staging slot
        if self._pending is not None:
            self._copied[self._pending % R].synchronize()
            self._pf.release(self._pending)
        self._pending = s
        self.bytes_copied += B * self._row_bytes

    def after_static_step(self) -> None:
        slot = self._s % self.slots
        self._consumed[slot].record(torch.cuda.current_stream())
        self._consumed_valid[slot] = True
        self._s += 1

    def gather_static(self) -> List[Tensor]:
        _lib.lib().gather_batch(self.ring, self.static, self._perm, self._cursor, self._arrive, self.batch_size, 0)
        return self.static

    def tail_batch(self) -> Optional[List[Tensor]]:
        idx = self._epoch_idx
        if idx is None:
            return None
        rest = idx[self._nfull * self.batch_size:]
        if rest.numel() == 0:
            return None
        return [t.index_select(0, rest).to(self.device) for t in self.host]

    def close(self) -> None:
        if self._pf is not None:
            self._pf.close()
            self._pf = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
