"""Backward-overlapped gradient sync hook (no imports of the ops: the op backwards call it).

An op's backward calls :func:`grad_ready` with gradient tensors (views of the flat gradient) the moment they are
final for the step; when a :class:`~masters_thesis_amd.parallel.ddp.FlatDDP` armed the overlapped sync for this
backward (``begin_backward``), their range is all-reduced on a side stream behind the rest of the backward
(reference: DDP's bucketed all-reduce fired by autograd hooks, `/root/reference/train.py:169-180`).
"""
from __future__ import annotations

ACTIVE = None  # the armed FlatDDP, or None


def grad_ready(*grads) -> None:
    if ACTIVE is not None:
        ACTIVE._ready(grads)
