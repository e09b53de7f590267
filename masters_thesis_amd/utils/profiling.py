"""Step tracing: per-phase device timers and an optional ``torch.profiler`` hook (SURVEY.md §5 "Tracing /
profiling"; the reference has none: `train.py:169-180` passes no ``profiler=``).

``Trainer(profiler="phases")`` runs the training steps eagerly (no HIP graph: a graph replay is one opaque
launch) and brackets every phase with a pair of HIP events on the compute stream:

    gather   batch assembly (device gather / streamed H2D hand-over)
    fwd      encoder forward (pipelined LSTM launch, or the extras' GEMM chain)
    loss     heads + loss + metrics (+ dh for the fused step)
    bwd      encoder backward (+ fused weight gradients)
    allreduce  gradient all-reduce (world > 1: xGMI one-shot or RCCL)
    optim    clip + Adam

Phases are marked with ``phase("name")`` from the engine and the models; the call is a no-op (one global
read) unless a timer is active, so the graph-captured production step pays nothing.  Per epoch the
trainer logs ``perf/phase/<name>_ms_p50`` (and ``perf/allreduce_us`` for world > 1).

``Trainer(profiler="torch")`` wraps the first ``profile_steps`` training steps of the first epoch in
``torch.profiler.profile`` (CPU + HIP activities) and writes a Chrome trace next to the logs.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional, Tuple

import torch

_ACTIVE: List[Optional["PhaseTimer"]] = [None]


def phase(name: str) -> None:
    """Start phase ``name`` (ends the previous one) on the active timer, if any."""
    t = _ACTIVE[0]
    if t is not None:
        t.mark(name)


class PhaseTimer:
    """Device-event phase timer.  ``begin_step`` / ``phase`` / ``end_step``; ``summarize`` syncs once."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self._steps: List[List[Tuple[str, object, object]]] = []
        self._cur: List[Tuple[str, object]] = []
        self._open: Optional[Tuple[str, object]] = None

    def _event(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        import time

        return time.perf_counter()

    def begin_step(self) -> None:
        self._cur = []
        self._open = None

    def mark(self, name: str) -> None:
        ev = self._event()
        if self._open is not None:
            self._cur.append((self._open[0], self._open[1], ev))
        self._open = (name, ev)

    def end_step(self) -> None:
        if self._open is not None:
            self._cur.append((self._open[0], self._open[1], self._event()))
            self._open = None
        if self._cur:
            self._steps.append(self._cur)
        self._cur = []

    def __enter__(self):
        _ACTIVE[0] = self
        return self

    def __exit__(self, *exc):
        _ACTIVE[0] = None
        return False

    def summarize(self, skip: int = 0) -> Dict[str, float]:
        """p50 ms per phase over the recorded steps (after ``skip`` warm-up steps)."""
        if self.cuda:
            torch.cuda.synchronize()
        per: Dict[str, List[float]] = {}
        steps = self._steps[skip:] if len(self._steps) > skip else self._steps
        for st in steps:
            acc: Dict[str, float] = {}
            for name, a, b in st:
                ms = a.elapsed_time(b) if self.cuda else (b - a) * 1e3
                acc[name] = acc.get(name, 0.0) + ms
            for k, v in acc.items():
                per.setdefault(k, []).append(v)
        out = {}
        for k, v in per.items():
            s = sorted(v)
            out[f"perf/phase/{k}_ms_p50"] = s[len(s) // 2]
        if "allreduce" in per:
            s = sorted(per["allreduce"])
            out["perf/allreduce_us"] = s[len(s) // 2] * 1e3
        self._steps = []
        return out


@contextlib.contextmanager
def torch_profile(trace_path: str, device: torch.device):
    """Profile the enclosed steps with ``torch.profiler`` and export a Chrome trace to ``trace_path``."""
    acts = [torch.profiler.ProfilerActivity.CPU]
    if device.type == "cuda":
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    prof.export_chrome_trace(trace_path)
