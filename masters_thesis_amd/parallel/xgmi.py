"""All-reduce over xGMI peer memory (``csrc/allreduce.hip``) for the flat gradient buckets.

Reference: Lightning's implicit DDP all-reduces the gradients with NCCL every step (`train.py:169-180`,
SURVEY §2.6 M2).  On one MI355X node the ranks are fully connected by xGMI (7 point-to-point links per GPU).
Every rank's comm buffer is mapped by every peer, so one kernel per bucket does the whole collective with no
host involvement (capturable inside the step's HIP graph):

* ONE-SHOT (buckets up to ``twoshot_kb``, default 512 KB: the LSTM's 204 KB bucket): every rank pushes the
  bucket into a slot of every peer (all links at once, one hop) and sums the N slots locally in rank order.
* TWO-SHOT (larger buckets: the transformer's 3.2 MB, mlp_large's 52 MB): reduce-scatter (chunk c to rank c)
  then all-gather of the reduced chunks -- each rank moves 2 (N-1)/N of the bucket instead of N-1 copies, over
  all 7 links in parallel (a ring uses one link per direction).

Each bucket is a range of the flat gradient with its own CHANNEL (epoch, counters, flags), so several buckets
can be in flight at once on different streams.

Setup (``XgmiAllReduce.create``) is collective-consistent: every rank allocates and exports its buffer, the
ranks agree on success (MIN all-reduce) before exchanging handles, open the peers' buffers, agree again, and on
any failure ALL ranks free what they hold and fall back together.  A self-check then compares the kernel
against the process group's own all-reduce (one- and two-shot, several rounds); any mismatch, exception or
timeout disables it (``FlatDDP`` keeps RCCL) and says why.  Waits are bounded and give-ups are counted in a
device word that ``check_health`` turns into an exception.

Selection (``MTA_ALLREDUCE``): ``auto`` (default: xGMI when all ranks share one node and the self-check
passes), ``xgmi`` (required: raise if unavailable), ``rccl``.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops._lib import lib

_LIVE: List["XgmiAllReduce"] = []
TWOSHOT_KB = 512.0  # buckets above this (and > 2 ranks) take the two-shot (reduce-scatter + all-gather) form


def _agree(ok: bool, device: torch.device, group) -> bool:
    """True on every rank iff ``ok`` on every rank (one MIN all-reduce all ranks take part in)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32,
                     device=device if dist.get_backend(group) == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item()) == 1


class XgmiAllReduce:
    def __init__(self, numel: int, device: torch.device, group=None, channels: int = 16):
        """Collective: every rank of ``group`` must construct it together.  Raises on failure on EVERY rank
        (after all of them released what they allocated)."""
        C = lib()
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.numel = int(numel)
        self.cap = -(-self.numel // 4) * 4
        self.channels = max(1, min(int(channels), int(C.xgmi_max_channels())))
        self.device = device
        self._C = C
        self.own = 0
        self._opened: List[int] = []
        self.bufs: List[int] = []
        err = ""
        handle = None
        try:  # local part first: allocation and export can fail on one rank only
            self.bytes = C.xgmi_buffer_bytes(self.world, self.cap, self.channels)
            self.own = C.xgmi_alloc(self.bytes)
            handle = C.xgmi_ipc_handle(self.own).tolist()
        except Exception as e:
            err = f"alloc/export: {e}"
        if not _agree(not err, device, group):
            self._release()
            raise RuntimeError(err or "alloc/export failed on another rank")
        handles = [None] * self.world
        dist.all_gather_object(handles, handle, group=group)
        try:
            for p, h in enumerate(handles):
                if p == self.rank:
                    self.bufs.append(self.own)
                else:
                    ptr = C.xgmi_ipc_open(torch.tensor(h, dtype=torch.uint8))
                    self.bufs.append(ptr)
                    self._opened.append(ptr)
            self.ctl = torch.zeros(C.xgmi_ctl_words(), dtype=torch.int32, device=device)
        except Exception as e:
            err = f"ipc open: {e}"
        if not _agree(not err, device, group):
            self._release()
            raise RuntimeError(err or "ipc open failed on another rank")
        self._timeout_word = int(C.xgmi_timeout_word())
        dist.barrier(group=group)  # every peer mapped every buffer before the first push
        _LIVE.append(self)

    # ------------------------------------------------------------------ use
    force_twoshot: Optional[bool] = None  # tests: exercise one form regardless of size / world

    def twoshot(self, numel: int) -> bool:
        if self.force_twoshot is not None:
            return self.force_twoshot
        return numel * 4 > TWOSHOT_KB * 1024 and self.world > 2

    def allreduce_(self, t: torch.Tensor, off: int = 0, channel: int = 0,
                   sq: Optional[torch.Tensor] = None) -> torch.Tensor:
        """In-place sum over the ranks of a contiguous fp32 CUDA tensor: the bucket [off, off + numel) of the flat
        gradient this object was sized for, on ``channel`` (concurrent buckets need distinct channels).  ``sq``
        (``xgmi_max_blocks()`` floats): the kernel's workgroups write the sums of squares of the reduced values
        there (the clip norm's partials, FusedAdam ``ext_norm``)."""
        if t.numel() % 4 or off % 4:
            raise ValueError("xgmi all-reduce needs 4-element-aligned buckets")
        self._C.xgmi_allreduce(t, int(off), self.cap, int(channel), self.channels, self.twoshot(t.numel()),
                               self.bufs, self.rank, self.ctl, sq)
        return t

    def timeouts(self) -> int:
        return int(self.ctl[self._timeout_word].item())

    def check_health(self) -> None:
        n = self.timeouts()
        if n:
            self.ctl[self._timeout_word].zero_()
            raise RuntimeError(f"xGMI all-reduce: {n} wait(s) on a peer gave up (that step's gradients are invalid)")

    def _release(self) -> None:
        try:
            torch.cuda.synchronize(self.device)
        except Exception:  # pragma: no cover
            pass
        for p in self._opened:
            try:
                self._C.xgmi_ipc_close(p)
            except Exception:  # pragma: no cover
                pass
        self._opened = []
        if self.own:
            try:
                self._C.xgmi_free(self.own)
            except Exception:  # pragma: no cover
                pass
            self.own = 0

    def close(self) -> None:
        if self in _LIVE:
            _LIVE.remove(self)
        self._release()

    # ------------------------------------------------------------------ construction + self-check
    @classmethod
    def create(cls, numel: int, device: torch.device, group=None, channels: int = 16) -> Optional["XgmiAllReduce"]:
        """The xGMI all-reduce for this group, or None on EVERY rank (with the reason printed once on rank 0) when
        the configuration does not allow it or its set-up / self-check fails anywhere."""
        mode = os.environ.get("MTA_ALLREDUCE", "auto").lower()
        if mode == "rccl":
            FALLBACK_REASON[0] = "MTA_ALLREDUCE=rccl"
            return None
        required = mode == "xgmi"

        def no(reason: str):
            FALLBACK_REASON[0] = reason
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
        try:
            ar = cls(numel, device, group, channels)
        except Exception as e:  # raised on every rank together
            return no(f"setup failed: {e}")
        ok, why = ar._self_check(group)
        if not _agree(ok, device, group):
            ar.close()
            return no(f"self-check failed: {why or 'on another rank'}")
        FALLBACK_REASON[0] = None
        return ar

    def _self_check(self, group, rounds: int = 3):
        g = torch.Generator(device=self.device).manual_seed(1234 + self.rank)
        sizes = sorted({min(self.cap, 1 << 12), min(self.cap, 1 << 20)})
        try:
            for form in (False, True):  # one-shot and two-shot, whatever the sizes would pick
                self.force_twoshot = form
                for n in sizes:
                    for r in range(rounds):
                        x = torch.randn(n, device=self.device, generator=g)
                        ref = x.clone()
                        dist.all_reduce(ref, group=group)
                        self.allreduce_(x, channel=r % self.channels)
                        torch.cuda.synchronize(self.device)
                        if self.timeouts():
                            return False, "peer wait timed out"
                        if not torch.allclose(x, ref, rtol=1e-5, atol=1e-5):
                            return False, (f"{'two' if form else 'one'}-shot n={n} round {r}: max err "
                                           f"{(x - ref).abs().max().item():.3g}")
            return True, ""
        except Exception as e:  # pragma: no cover - surfaced through the MIN all-reduce
            return False, str(e)
        finally:
            self.force_twoshot = None


# why the last XgmiAllReduce.create returned None (the bench record's allreduce_fallback_reason), None after a success
FALLBACK_REASON: List[Optional[str]] = [None]


def check_all_health() -> None:
    for ar in list(_LIVE):
        ar.check_health()
