"""``LightningModule``-compatible base class ("Lightning Trainer").

Keeps the reference model code shape (`src/model.py`): ``save_hyperparameters()``,
``self.hparams``, ``self.log(name, value_or_metric, on_step, on_epoch)``,
``training_step`` / ``validation_step`` / ``test_step``, ``configure_optimizers``,
``on_test_start`` / ``on_test_end`` and ``Cls.load_from_checkpoint(path, map_location)``.

Logging is device-resident: a tensor logged with ``on_epoch=True`` feeds a
batch-size-weighted ``MeanAccumulator``; a logged ``Metric`` object is computed at
epoch end.  Nothing calls ``.item()`` per step, so the whole step (including the
logging) replays from a HIP graph.
"""
from __future__ import annotations

import inspect
from typing import Any, Dict, Optional

import torch

from ..metrics import MeanAccumulator, Metric


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class LightningModule(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self._hparams = AttributeDict()
        self._hparams_name = "kwargs"
        self.trainer = None
        self._stage = "train"
        self._current_batch_size = 1
        # per-stage {name: Metric}
        self._epoch_logs: Dict[str, Dict[str, Metric]] = {"train": {}, "val": {}, "test": {}}
        self._compiled = False

    # ---- hyper-parameters ----------------------------------------------------
    def save_hyperparameters(self, *names, ignore=None) -> None:
        frame = inspect.currentframe().f_back
        init = type(self).__init__
        sig = inspect.signature(init)
        ignore = set([ignore] if isinstance(ignore, str) else (ignore or []))
        hp = {}
        for pname, p in sig.parameters.items():
            if pname == "self" or p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD) or pname in ignore:
                continue
            if names and pname not in names:
                continue
            if pname in frame.f_locals:
                hp[pname] = frame.f_locals[pname]
        self._hparams.update(hp)

    @property
    def hparams(self) -> AttributeDict:
        return self._hparams

    # ---- logging ------------------------------------------------------------------
    def log(self, name: str, value: Any, on_step: bool = False, on_epoch: bool = True, prog_bar: bool = False,
            sync_dist: bool = False, batch_size: Optional[int] = None, **_) -> None:
        if not on_epoch:
            return
        logs = self._epoch_logs[self._stage]
        if isinstance(value, Metric):
            logs[name] = value
            return
        acc = logs.get(name)
        if acc is None or not isinstance(acc, MeanAccumulator):
            acc = MeanAccumulator().to(value.device if torch.is_tensor(value) else "cpu")
            logs[name] = acc
        v = value if torch.is_tensor(value) else torch.tensor(float(value))
        acc.update(v, float(batch_size or self._current_batch_size))

    def logged_metrics(self, stage: str) -> Dict[str, Metric]:
        return self._epoch_logs[stage]

    # ---- hooks (overridable) -------------------------------------------------------
    def training_step(self, batch, batch_idx):  # pragma: no cover - abstract
        raise NotImplementedError

    def validation_step(self, batch, batch_idx):
        return None

    def test_step(self, batch, batch_idx):
        return None

    def on_test_start(self):
        pass

    def on_test_end(self):
        pass

    def on_train_epoch_start(self):
        pass

    def on_train_epoch_end(self):
        pass

    def configure_optimizers(self):  # pragma: no cover - abstract
        raise NotImplementedError

    def compile(self, *args, **kwargs):
        """The reference calls ``model.compile()`` (`train.py:137`).  Here the hot path is
        already fused HIP kernels replayed from a HIP graph, so this only records the request."""
        self._compiled = True
        return self

    # ---- checkpoint helpers ----------------------------------------------------------
    def on_save_checkpoint(self, checkpoint: Dict[str, Any]) -> None:
        pass

    def on_load_checkpoint(self, checkpoint: Dict[str, Any]) -> None:
        pass

    @classmethod
    def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict: bool = True, **kwargs):
        from .checkpoint import load_checkpoint

        ckpt = load_checkpoint(checkpoint_path, map_location=map_location)
        hp = dict(ckpt.get("hyper_parameters", {}))
        hp.update(kwargs)
        model = cls(**hp)
        model.on_load_checkpoint(ckpt)
        model.load_state_dict(ckpt["state_dict"], strict=strict)
        if map_location is not None and not callable(map_location):
            model.to(map_location)
        return model
