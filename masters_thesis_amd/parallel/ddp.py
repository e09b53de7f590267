"""Data-parallel gradient synchronisation over the flat gradient buffer.

Reference: Lightning's implicit DDP — a 25 MB reducer bucket, i.e. ONE all-reduce
of the whole 0.2-1.0 MB fp32 gradient per step.

MI355X design: gradients already live in one contiguous buffer
(``ops.optim.FlatParameters``), so the all-reduce is issued directly on it (no
bucket copy-in/copy-out).  The average's 1/world factor is folded into the fused
clip+Adam kernel (``grad_scale``) instead of a separate division kernel.  For large
models (the MLP/transformer extras) the buffer is split into ``bucket_mb`` chunks;
xGMI is point-to-point (7 links x ~153 GB/s), so a ring all-reduce is per-link
bound and a few large buckets beat many small ones — the default bucket is 64 MB,
and buckets are issued asynchronously so RCCL can pipeline them.

On one node every bucket goes through the xGMI all-reduce instead (``parallel/xgmi.py``: one kernel per
bucket, one-shot for small buckets, reduce-scatter + all-gather over all 7 links for large ones, summed in rank
order), which is also safe to capture inside the step's HIP graph (``graph_safe``), so grouped multi-step
graphs stay on for world > 1 whatever the model size; ``MTA_ALLREDUCE=rccl`` keeps RCCL (eager, after the
captured backward).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops.optim import FlatParameters
from . import overlap as _ov
from .overlap import grad_ready  # noqa: F401  (re-export)


class FlatDDP:
    def __init__(self, flat: FlatParameters, group=None, bucket_mb: float = 64.0):
        self.flat = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        n = flat.padded
        per = max(1024, int(bucket_mb * (1 << 20) / 4) // 1024 * 1024)
        self.buckets: List[slice] = [slice(i, min(i + per, n)) for i in range(0, n, per)]
        self._gloo_cpu = self.world > 1 and dist.get_backend(group) == "gloo" and flat.grad.is_cuda
        # one-shot xGMI all-reduce (csrc/allreduce.hip) for single-node GPU groups; None -> the group's all-reduce
        self.xgmi = None
        # GPU gradients: the xGMI kernel whatever the host process group is (RCCL, or gloo when ranks share a GPU);
        # XgmiAllReduce.create returns None (-> the group's all-reduce) under MTA_ALLREDUCE=rccl or a failed check
        if self.world > 1 and flat.grad.is_cuda:
            from .xgmi import XgmiAllReduce

            self.xgmi = XgmiAllReduce.create(flat.padded, flat.grad.device, group)
        # xGMI buckets (4-float aligned ranges of the flat gradient, one channel each)
        xper = max(4096, int(float(os.environ.get("MTA_XGMI_BUCKET_MB", "64")) * (1 << 20) / 4) // 4096 * 4096)
        self.xgmi_buckets: List[slice] = [slice(i, min(i + xper, n)) for i in range(0, n, xper)]

        # backward-overlapped sync (xGMI only: a plain kernel, capturable on a side stream): ranges of the flat
        # gradient reported final by grad_ready() during the backward are reduced there as they come
        self.overlap = (self.xgmi is not None and os.environ.get("MTA_DDP_OVERLAP", "1") != "0")
        self.overlap_min_bytes = int(float(os.environ.get("MTA_DDP_OVERLAP_MIN_KB", "256")) * 1024)
        self._side: Optional[torch.cuda.Stream] = None
        self._done: List[tuple] = []     # [start, stop) ranges already all-reduced this step
        self._pending: List[tuple] = []  # ready ranges not yet launched (below the minimum size)
        self._launches = 0
        self._reduce_fn = None           # tests: replaces the xGMI launch (range -> None)
        # range -> channel, fixed for the life of this object.  csrc/allreduce.hip's parity double buffer protects
        # consecutive calls of ONE channel only (inbox slots are indexed by flat offset, shared by all channels): a
        # range reduced on channel c1 in one step and c2 in the next could let a fast peer overwrite a slot a slow
        # rank is still reading.  So a range keeps the channel it was first given, in eager steps and
        # (captured once) in graph replays alike.
        self._chan_of: dict = {}
        self._plan: List[tuple] = []      # the ranges of the last overlapped step, in launch order
        # clip-norm partials of the reduced gradient (xGMI only): every range reduced in a step writes the squares of
        # its reduced values into a slot of its own (fixed per range, like its channel), so the fused optimizer takes
        # the norm from here (``norm_parts``) and the weight-gradient producers stay on with world > 1
        self.sq: Optional[torch.Tensor] = None
        self._sq_of: dict = {}
        if self.xgmi is not None:
            from ..ops._lib import lib

            self._sq_block = int(lib().xgmi_max_blocks())
            self.sq = torch.zeros(self.SQ_SLOTS * self._sq_block, device=flat.grad.device, dtype=torch.float32)

    SQ_SLOTS = 256  # ranges per step with a norm-partials slot of their own

    @property
    def norm_parts(self) -> Optional[torch.Tensor]:
        """The clip-norm partials of the whole reduced gradient (FusedAdam.step ``ext_norm``), or None when this
        sync does not produce them (world 1, the process group's all-reduce, a test's replacement launch)."""
        return self.sq if (self.xgmi is not None and self._reduce_fn is None) else None

    def _sq_slot(self, a: int, b: int) -> Optional[torch.Tensor]:
        if self.sq is None:
            return None
        k = self._sq_of.get((a, b))
        if k is None:
            k = len(self._sq_of)
            if k >= self.SQ_SLOTS:
                raise RuntimeError(f"more than {self.SQ_SLOTS} all-reduce ranges per step: raise FlatDDP.SQ_SLOTS")
            self._sq_of[(a, b)] = k
        return self.sq[k * self._sq_block:(k + 1) * self._sq_block]

    def _xg(self, g: torch.Tensor, a: int, b: int, channel: int) -> None:
        self.xgmi.allreduce_(g[a:b], off=a, channel=channel, sq=self._sq_slot(a, b))

    # ------------------------------------------------------------------ overlapped sync
    def begin_backward(self) -> None:
        """Arm grad_ready() for the coming backward (call before it; allreduce_grads() disarms)."""
        self._done, self._pending, self._launches = [], [], 0
        if self.overlap or self._reduce_fn is not None:
            _ov.ACTIVE = self

    def _range_of(self, t: torch.Tensor) -> Optional[tuple]:
        g = self.flat.grad
        if t is None or t.device != g.device or t.dtype != g.dtype or not t.is_contiguous():
            return None
        off = (t.data_ptr() - g.data_ptr()) // g.element_size()
        if off < 0 or off + t.numel() > g.numel():
            return None
        return (off, off + t.numel())

    def _ready(self, grads) -> None:
        rs = sorted(r for r in (self._range_of(t) for t in grads) if r is not None)
        for r in rs:
            self._pending.append(r)
        self._pending.sort()
        merged: List[tuple] = []
        for a, b in self._pending:
            if merged and merged[-1][1] == a:
                merged[-1] = (merged[-1][0], b)
            else:
                merged.append((a, b))
        self._pending = []
        for a, b in merged:
            # 4-float-aligned interior goes now if it is big enough; the rest waits for the final sync
            a4, b4 = -(-a // 4) * 4, b // 4 * 4
            if (b4 - a4) * 4 >= self.overlap_min_bytes:
                self._launch(a4, b4, side=True)
                if a4 > a:
                    self._pending.append((a, a4))
                if b > b4:
                    self._pending.append((b4, b))
            else:
                self._pending.append((a, b))

    def channel_of(self, a: int, b: int) -> int:
        """The channel of range [a, b): assigned on first use, then never changed.  Every gradient element belongs to
        ONE registered range for the life of this object (a range overlapping a different registered one raises):
        that is what makes the per-channel parity double buffer sufficient."""
        ch = self._chan_of.get((a, b))
        if ch is None:
            for (a2, b2) in self._chan_of:
                if a < b2 and a2 < b:
                    raise RuntimeError(f"xGMI channel invariant: range [{a}, {b}) overlaps the registered range "
                                       f"[{a2}, {b2}) (the backward's ready ranges changed between steps)")
            nch = self.xgmi.channels if self.xgmi is not None else 16
            ch = len(self._chan_of) % nch
            self._chan_of[(a, b)] = ch
        return ch

    def _launch(self, a: int, b: int, side: bool) -> None:
        self._done.append((a, b))
        self._launches += 1
        if self._reduce_fn is not None:
            self._reduce_fn(a, b)
            return
        k = self.channel_of(a, b)
        g = self.flat.grad
        if side:
            if self._side is None:
                self._side = torch.cuda.Stream(device=g.device)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(g.device))
            self._side.wait_event(ev)
            with torch.cuda.stream(self._side):
                self._xg(g, a, b, k)
        else:
            self._xg(g, a, b, k)

    def _remaining(self, n: int) -> List[tuple]:
        """[0, n) minus the ranges already reduced, in order."""
        out, cur = [], 0
        for a, b in sorted(self._done):
            if a > cur:
                out.append((cur, a))
            cur = max(cur, b)
        if cur < n:
            out.append((cur, n))
        return out

    @property
    def backend_name(self) -> str:
        if self.world == 1:
            return "none"
        return "xgmi" if self.xgmi is not None else dist.get_backend(self.group)

    @property
    def fallback_reason(self):
        """Why the gradient all-reduce is the process group's rather than the xGMI kernel (None when xGMI runs or
        world == 1): the configuration check, the set-up error or the failed self-check round."""
        if self.world == 1 or self.xgmi is not None:
            return None
        from .xgmi import FALLBACK_REASON

        return FALLBACK_REASON[0] or "xGMI all-reduce not attempted (no GPU process group or not on one node)"

    @property
    def graph_safe(self) -> bool:
        """The gradient sync can live inside the captured step graph (a plain kernel: xGMI one-shot)."""
        return self.world == 1 or self.xgmi is not None

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.world

    def broadcast_parameters(self, src: int = 0) -> None:
        """DDP construction-time parameter broadcast."""
        if self.world == 1:
            return
        if self._gloo_cpu:
            t = self.flat.data.cpu()
            dist.broadcast(t, src=src, group=self.group)
            self.flat.data.copy_(t)
        else:
            dist.broadcast(self.flat.data, src=src, group=self.group)

    def allreduce_grads(self) -> None:
        """Sum gradients across ranks (the mean's 1/world is applied by the optimizer)."""
        if self.world == 1:
            return
        g = self.flat.grad
        if _ov.ACTIVE is self:
            # overlapped: the rest of the buffer (xGMI-bucket-sized pieces) on the main stream, then join the side
            # stream so the optimizer sees every reduced range
            # (joined first: a channel is only ever reused in stream order)
            _ov.ACTIVE = None
            if self._side is not None and self._reduce_fn is None:
                torch.cuda.current_stream(g.device).wait_stream(self._side)
            xper = self.xgmi_buckets[0].stop - self.xgmi_buckets[0].start if self.xgmi_buckets else g.numel()
            for a, b in self._remaining(g.numel()):
                for s0 in range(a, b, xper):
                    self._launch(s0, min(b, s0 + xper), side=False)
            self._plan = list(self._done)
            return
        if self.xgmi is not None:
            if self._chan_of and self._plan:
                # an un-armed sync after overlapped steps (bench.py's allreduce_us loop): the same ranges on the same
                # channels as those steps, in stream order
                for a, b in self._plan:
                    self._xg(g, a, b, self.channel_of(a, b))
                return
            for b in self.xgmi_buckets:
                self._xg(g, b.start, b.stop, self.channel_of(b.start, b.stop))
            return
        if self._gloo_cpu:
            t = g.cpu()
            dist.all_reduce(t, group=self.group)
            g.copy_(t)
            return
        if len(self.buckets) == 1:
            dist.all_reduce(g, group=self.group)
            return
        works = [dist.all_reduce(g[b], group=self.group, async_op=True) for b in self.buckets]
        for w in works:
            w.wait()
