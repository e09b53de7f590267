"""``ReduceLROnPlateau`` for the fused optimizer (reference: `src/model.py:156-172`).

Identical decision rule to ``torch.optim.lr_scheduler.ReduceLROnPlateau``
(mode, factor, patience, threshold/rel, cooldown, min_lr, eps); it writes the new
lr into the optimizer's device scalar, so a captured train-step graph picks it up
without re-capture.
"""
from __future__ import annotations

import math
from typing import Any, Dict


class PlateauScheduler:
    def __init__(self, optimizer, mode: str = "min", factor: float = 0.1, patience: int = 10,
                 threshold: float = 1e-4, threshold_mode: str = "rel", cooldown: int = 0, min_lr: float = 0.0,
                 eps: float = 1e-8):
        if factor >= 1.0:
            raise ValueError("factor should be < 1.0")
        self.optimizer = optimizer
        self.mode, self.factor, self.patience = mode, factor, patience
        self.threshold, self.threshold_mode = threshold, threshold_mode
        self.cooldown, self.min_lr, self.eps = cooldown, float(min_lr), eps
        self.best = math.inf if mode == "min" else -math.inf
        self.num_bad_epochs = 0
        self.cooldown_counter = 0
        self.last_epoch = 0
        self._last_lr = [optimizer.lr]

    @classmethod
    def from_torch(cls, sched, optimizer) -> "PlateauScheduler":
        ml = sched.min_lrs[0] if hasattr(sched, "min_lrs") else 0.0
        return cls(optimizer, mode=sched.mode, factor=sched.factor, patience=sched.patience,
                   threshold=sched.threshold, threshold_mode=sched.threshold_mode, cooldown=sched.cooldown,
                   min_lr=ml, eps=sched.eps)

    def is_better(self, a: float, best: float) -> bool:
        if self.mode == "min" and self.threshold_mode == "rel":
            return a < best * (1.0 - self.threshold)
        if self.mode == "min":
            return a < best - self.threshold
        if self.threshold_mode == "rel":
            return a > best * (self.threshold + 1.0)
        return a > best + self.threshold

    def step(self, metric: float) -> None:
        current = float(metric)
        self.last_epoch += 1
        if self.is_better(current, self.best):
            self.best = current
            self.num_bad_epochs = 0
        else:
            self.num_bad_epochs += 1
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.num_bad_epochs = 0
        if self.num_bad_epochs > self.patience:
            old = self.optimizer.lr
            new = max(old * self.factor, self.min_lr)
            if old - new > self.eps:
                self.optimizer.set_lr(new)
            self.cooldown_counter = self.cooldown
            self.num_bad_epochs = 0
        self._last_lr = [self.optimizer.lr]

    def get_last_lr(self):
        return list(self._last_lr)

    def state_dict(self) -> Dict[str, Any]:
        return {k: v for k, v in self.__dict__.items() if k != "optimizer"}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        self.__dict__.update(sd)
