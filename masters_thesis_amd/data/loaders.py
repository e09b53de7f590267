"""Batch loaders over window tensors (replaces the reference's ``torch.utils.data.DataLoader``s,
`src/data.py:236-244`).

``TensorBatchLoader`` walks rows ``[start, stop)`` of a list of same-length tensors in
``batch_size`` chunks, reshuffled per epoch from ``seed + epoch`` and sharded over ranks
(rank r takes positions r, r + world, ... of the epoch order; the train split is trimmed to
a multiple of ``world`` so every rank runs the same number of steps, evaluation splits are
not padded: metrics are summed across ranks, so duplicated windows would bias them).

When the tensors live in HBM the loader also offers the *static* protocol used by the
engine's captured step graphs:

* ``begin_epoch(e)`` uploads the epoch order to a device permutation buffer, resets the device
  cursor and returns the number of full batches;
* ``gather_static()`` launches ``csrc/lstm_aux.hip::gather_batch_kernel`` which copies rows
  ``perm[cursor·B : (cursor+1)·B]`` into fixed batch buffers and advances the cursor on the
  device — so one captured graph replays every step of every epoch with no host work;
* ``tail_batch()`` returns the last partial batch (``drop_last=False`` semantics) eagerly.
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Sequence

import torch
from torch import Tensor

from ..ops import _lib


class TensorBatchLoader:
    def __init__(self, tensors: Sequence[Tensor], batch_size: int, shuffle: bool = False, seed: int = 0,
                 rank: int = 0, world_size: int = 1, start: int = 0, stop: Optional[int] = None,
                 even_shards: Optional[bool] = None):
        self.tensors: List[Tensor] = list(tensors)
        if not self.tensors:
            raise ValueError("TensorBatchLoader needs at least one tensor")
        n = int(self.tensors[0].shape[0])
        if any(int(t.shape[0]) != n for t in self.tensors):
            raise ValueError("all tensors must have the same number of rows")
        self.start = int(start)
        self.stop = n if stop is None else int(stop)
        if not 0 <= self.start <= self.stop <= n:
            raise ValueError(f"bad row range [{self.start}, {self.stop}) for {n} rows")
        self.batch_size = int(batch_size)
        if self.batch_size < 1:
            raise ValueError("batch_size must be >= 1")
        self.shuffle = bool(shuffle)
        self.seed = int(seed)
        self.rank, self.world_size = int(rank), int(world_size)
        # training shards must have equal step counts (collectives every step); eval shards need not
        self.even_shards = self.shuffle if even_shards is None else bool(even_shards)
        self.epoch = 0
        self.device = self.tensors[0].device
        self._epoch_idx: Optional[Tensor] = None
        self._perm = self._cursor = self._arrive = None
        self._static: Optional[List[Tensor]] = None
        self._nfull = 0

    # ------------------------------------------------------------------ order
    @property
    def n_rows(self) -> int:
        return self.stop - self.start

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def epoch_indices(self, epoch: Optional[int] = None) -> Tensor:
        """Absolute row indices this rank visits in ``epoch`` (CPU int64)."""
        e = self.epoch if epoch is None else int(epoch)
        if self.shuffle:
            g = torch.Generator().manual_seed(self.seed + e)
            order = torch.randperm(self.n_rows, generator=g)
        else:
            order = torch.arange(self.n_rows)
        if self.world_size > 1:
            if self.even_shards:
                order = order[: (self.n_rows // self.world_size) * self.world_size]
            order = order[self.rank::self.world_size]
        return order + self.start

    def _rows_per_rank(self) -> int:
        if self.world_size == 1:
            return self.n_rows
        if self.even_shards:
            return self.n_rows // self.world_size
        return len(range(self.rank, self.n_rows, self.world_size))

    def __len__(self) -> int:
        return -(-self._rows_per_rank() // self.batch_size)

    def _select(self, rows: Tensor) -> List[Tensor]:
        rows = rows.to(self.device)
        return [t.index_select(0, rows) for t in self.tensors]

    def __iter__(self) -> Iterator[List[Tensor]]:
        idx = self.epoch_indices()
        for i in range(0, idx.numel(), self.batch_size):
            yield self._select(idx[i:i + self.batch_size])

    # ------------------------------------------------------------------ static (in-graph gather) protocol
    def supports_static(self) -> bool:
        return (self.device.type == "cuda" and len(self.tensors) <= 4
                and all(t.dtype == torch.float32 and t.is_contiguous() for t in self.tensors)
                and _lib.use_hip(self.tensors[0]))

    def _ensure_static(self) -> None:
        if self._static is not None:
            return
        dev = self.device
        self._static = [torch.empty((self.batch_size, *t.shape[1:]), dtype=t.dtype, device=dev)
                        for t in self.tensors]
        self._perm = torch.zeros(max(self._rows_per_rank(), 1), dtype=torch.int32, device=dev)
        self._cursor = torch.zeros(1, dtype=torch.int32, device=dev)
        self._arrive = torch.zeros(65 * 32, dtype=torch.int32, device=dev)  # gather arrival counters, one line each

    def begin_epoch(self, epoch: int) -> int:
        self._ensure_static()
        self.set_epoch(epoch)
        idx = self.epoch_indices()
        self._epoch_idx = idx
        if idx.numel():
            self._perm[: idx.numel()].copy_(idx.to(torch.int32))
        self._cursor.zero_()
        self._arrive.zero_()
        self._nfull = idx.numel() // self.batch_size
        return self._nfull

    def gather_static(self, defer: bool = False) -> List[Tensor]:
        """Next batch in the static buffers (device gather, cursor advanced on the device).

        ``defer``: launch nothing and return a :class:`DeferredBatch` — the consumer (the pipelined LSTM forward
        of the fused training step) reads the rows through the permutation and fills the buffers itself, or
        calls ``materialize()`` to run the gather kernel."""
        if defer:
            return DeferredBatch(self)
        _lib.lib().gather_batch(self.tensors, self._static, self._perm, self._cursor, self._arrive,
                                self.batch_size, 0)
        return self._static

    def tail_batch(self) -> Optional[List[Tensor]]:
        idx = self._epoch_idx
        rest = idx[self._nfull * self.batch_size:] if idx is not None else idx
        if rest is None or rest.numel() == 0:
            return None
        return self._select(rest)


class DeferredBatch(list):
    """The static batch buffers of a loader whose gather has not run yet (``gather_static(defer=True)``).

    ``gather_args()`` gives what a kernel needs to fold the gather in (source tensors, static buffers,
    permutation, cursor, windows per batch); a consumer that does so calls ``consumed()``; any other consumer must
    call ``materialize()`` first."""

    def __init__(self, loader):
        super().__init__(loader._static)
        self._loader = loader
        self.pending = True

    def gather_args(self):
        ld = self._loader
        return list(ld.tensors), list(ld._static), ld._perm, ld._cursor, ld.batch_size

    def consumed(self) -> None:
        self.pending = False

    def materialize(self) -> "DeferredBatch":
        if self.pending:
            ld = self._loader
            _lib.lib().gather_batch(ld.tensors, ld._static, ld._perm, ld._cursor, ld._arrive, ld.batch_size, 0)
            self.pending = False
        return self

