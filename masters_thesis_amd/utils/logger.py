"""TensorBoard-compatible experiment logger (Lightning ``TensorBoardLogger`` contract).

Same directory layout as the reference (`train.py:143-148`, `configs/config.yaml:9-13`):
``<save_dir>/<name>/<version>/events.out.tfevents.*`` plus ``hparams.yaml``; the
checkpoint callback writes ``<save_dir>/<name>/<version>/checkpoints``.
Every scalar is mirrored to ``metrics.jsonl`` for tooling.  Only global rank 0
writes (the others get a no-op logger).
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path
from typing import Any, Dict, Mapping, Optional

import yaml

from .tfevents import EventFileWriter


def _flatten(d: Mapping, prefix: str = "", sep: str = "/") -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for k, v in d.items():
        key = f"{prefix}{sep}{k}" if prefix else str(k)
        if isinstance(v, Mapping):
            out.update(_flatten(v, key, sep))
        else:
            out[key] = v
    return out


def _sanitize(v: Any) -> Any:
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    try:
        import torch

        if isinstance(v, torch.Tensor) and v.numel() == 1:
            return v.item()
    except Exception:  # pragma: no cover
        pass
    return str(v)


class _Experiment:
    """Subset of ``SummaryWriter`` used by the reference (`test.py:91-145`, `src/plots.py:76`)."""

    def __init__(self, writer: Optional[EventFileWriter]):
        self._w = writer

    def add_scalar(self, tag, value, global_step=0):
        if self._w:
            self._w.add_scalar(tag, float(value), int(global_step or 0))

    def add_figure(self, tag, figure, global_step=0, close=True):
        if self._w:
            self._w.add_figure(tag, figure, int(global_step or 0), close)
        else:  # still close to free memory on non-zero ranks
            import matplotlib.pyplot as plt

            plt.close(figure)

    def flush(self):
        if self._w:
            self._w.flush()

    def close(self):
        if self._w:
            self._w.close()


class TensorBoardLogger:
    def __init__(self, save_dir: os.PathLike, name: str = "lightning_logs", version: Optional[str] = None,
                 default_hp_metric: bool = True, rank: int = 0):
        self.save_dir = str(save_dir)
        self.name = str(name)
        self._version = version
        self.default_hp_metric = default_hp_metric
        self.rank = rank
        self._writer: Optional[EventFileWriter] = None
        self._hparams: Dict[str, Any] = {}
        self._jsonl = None

    @property
    def version(self) -> str:
        if self._version is None:
            root = Path(self.save_dir) / self.name
            existing = [int(p.name.split("_")[1]) for p in root.glob("version_*") if p.name.split("_")[1].isdigit()] \
                if root.exists() else []
            self._version = f"version_{max(existing) + 1 if existing else 0}"
        return str(self._version)

    @property
    def log_dir(self) -> str:
        return str(Path(self.save_dir) / self.name / self.version)

    @property
    def experiment(self) -> _Experiment:
        if self.rank == 0 and self._writer is None:
            self._writer = EventFileWriter(self.log_dir)
            self._jsonl = open(Path(self.log_dir) / "metrics.jsonl", "a")
            if self.default_hp_metric:
                self._writer.add_scalar("hp_metric", -1, 0)
        return _Experiment(self._writer)

    def log_metrics(self, metrics: Mapping[str, float], step: int) -> None:
        exp = self.experiment
        if self.rank != 0:
            return
        rec = {"step": int(step), "time": time.time()}
        for k, v in metrics.items():
            v = float(v)
            exp.add_scalar(k, v, step)
            rec[k] = v
        self._jsonl.write(json.dumps(rec) + "\n")
        self._jsonl.flush()

    def log_hyperparams(self, params: Mapping[str, Any], metrics: Optional[Mapping[str, float]] = None) -> None:
        self.experiment
        if self.rank != 0:
            return
        flat = {k: _sanitize(v) for k, v in _flatten(dict(params)).items()}
        self._hparams.update(flat)
        self.save()
        if metrics:
            self._writer.add_hparams(flat, {k: float(v) for k, v in metrics.items()}, 0)
            self._jsonl.write(json.dumps({"hparams_metrics": {k: float(v) for k, v in metrics.items()}}) + "\n")
            self._jsonl.flush()

    def save(self) -> None:
        if self.rank != 0:
            return
        Path(self.log_dir).mkdir(parents=True, exist_ok=True)
        with open(Path(self.log_dir) / "hparams.yaml", "w") as f:
            yaml.safe_dump(self._hparams, f, sort_keys=False)

    def finalize(self) -> None:
        if self._writer:
            self._writer.flush()
        if self._jsonl:
            self._jsonl.flush()

    def close(self) -> None:
        if self._writer:
            self._writer.close()
        if self._jsonl:
            self._jsonl.close()
