"""Trainer callbacks: ModelCheckpoint, LearningRateMonitor, EarlyStopping, StepTimer.

``ModelCheckpoint`` reproduces the reference configuration (`train.py:151-161`):
``dirpath=<save_dir>/<name>/<version>/checkpoints``,
``filename="best_epoch={epoch:02d}_val={loss/total/val:.4f}"``, ``monitor="loss/total/val"``,
``mode="min"``, ``save_last=True``, ``auto_insert_metric_name=False`` -> files
``best_epoch=03_val=1.2345.ckpt`` (top-1, older best removed) and ``last.ckpt``.
``LearningRateMonitor(logging_interval="epoch")`` logs ``lr-Adam`` (`train.py:162-165`).
``EarlyStopping`` is the thesis' patience-10 stopping (`tex/diplomski_rad.tex:1126`,
SURVEY Q16), off unless configured.
"""
from __future__ import annotations

import math
import re
import time
from pathlib import Path
from typing import Any, Dict, List, Optional

import torch


class Callback:
    def on_fit_start(self, trainer, module):
        pass

    def on_train_epoch_start(self, trainer, module):
        pass

    def on_train_epoch_end(self, trainer, module):
        pass

    def on_validation_end(self, trainer, module):
        pass

    def on_fit_end(self, trainer, module):
        pass

    def on_test_end(self, trainer, module):
        pass

    def state_dict(self) -> Dict[str, Any]:
        return {}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        pass

    @property
    def state_key(self) -> str:
        return type(self).__name__


def format_checkpoint_name(filename: str, metrics: Dict[str, Any], auto_insert_metric_name: bool = True) -> str:
    groups = re.findall(r"(\{.*?)[:\}]", filename)
    groups = sorted(groups, key=len, reverse=True)
    metrics = dict(metrics)
    for group in groups:
        name = group[1:]
        if auto_insert_metric_name:
            filename = filename.replace(group, name.replace("/", "_") + "={" + name)
        filename = filename.replace(group, "{0[" + name + "]")
        if name not in metrics:
            metrics[name] = 0
    vals = {k: (float(v) if torch.is_tensor(v) and v.is_floating_point() else
                int(v) if torch.is_tensor(v) else v) for k, v in metrics.items()}
    return filename.format(vals)


class ModelCheckpoint(Callback):
    def __init__(self, dirpath: Optional[str] = None, filename: Optional[str] = None, monitor: Optional[str] = None,
                 mode: str = "min", save_last: Optional[bool] = None, save_top_k: int = 1,
                 auto_insert_metric_name: bool = True, every_n_epochs: int = 1):
        self.dirpath = dirpath
        self.filename = filename or "{epoch}-{step}"
        self.monitor = monitor
        self.mode = mode
        self.save_last = save_last
        self.save_top_k = save_top_k
        self.auto_insert_metric_name = auto_insert_metric_name
        self.every_n_epochs = every_n_epochs
        self.best_model_path = ""
        self.best_model_score: Optional[torch.Tensor] = None
        self.last_model_path = ""
        self._last_saved_epoch = -1

    @property
    def state_key(self) -> str:
        return f"ModelCheckpoint{{'monitor': {self.monitor!r}, 'mode': {self.mode!r}}}"

    def _better(self, cur: float) -> bool:
        if self.best_model_score is None:
            return True
        best = float(self.best_model_score)
        return cur < best if self.mode == "min" else cur > best

    def _save_all(self, trainer, module) -> None:
        if trainer.sanity_checking or self._last_saved_epoch == trainer.current_epoch:
            return
        metrics = dict(trainer.callback_metrics)
        metrics["epoch"] = trainer.current_epoch
        metrics["step"] = trainer.global_step
        d = Path(self.dirpath or Path(trainer.default_root_dir) / "checkpoints")
        saved = False
        if self.monitor is None or self.monitor in metrics:
            cur = float(metrics[self.monitor]) if self.monitor else float(trainer.current_epoch)
            if self.monitor is None or (not math.isnan(cur) and self._better(cur)):
                name = format_checkpoint_name(self.filename, metrics, self.auto_insert_metric_name)
                path = d / f"{name}.ckpt"
                v = 1
                while path.exists() and str(path) != self.best_model_path:
                    path = d / f"{name}-v{v}.ckpt"
                    v += 1
                old = self.best_model_path
                self.best_model_score = torch.tensor(cur)
                self.best_model_path = str(path)
                trainer.save_checkpoint(path)
                saved = True
                if old and old != str(path) and self.save_top_k == 1 and trainer.is_global_zero:
                    Path(old).unlink(missing_ok=True)
        if self.save_last:
            last = d / "last.ckpt"
            trainer.save_checkpoint(last)
            self.last_model_path = str(last)
            saved = True
        if saved:
            self._last_saved_epoch = trainer.current_epoch

    def _should_save_on_train_epoch_end(self, trainer) -> bool:
        if trainer.check_val_every_n_epoch != 1:
            return False
        return trainer.num_val_batches == 0

    def on_validation_end(self, trainer, module):
        self._save_all(trainer, module)

    def on_train_epoch_end(self, trainer, module):
        if self._should_save_on_train_epoch_end(trainer):
            self._save_all(trainer, module)

    def state_dict(self):
        return {"monitor": self.monitor, "best_model_score": self.best_model_score,
                "best_model_path": self.best_model_path, "last_model_path": self.last_model_path,
                "dirpath": str(self.dirpath)}

    def load_state_dict(self, sd):
        self.best_model_score = sd.get("best_model_score")
        self.best_model_path = sd.get("best_model_path", "")
        self.last_model_path = sd.get("last_model_path", "")


class LearningRateMonitor(Callback):
    def __init__(self, logging_interval: Optional[str] = "epoch", log_momentum: bool = False):
        self.logging_interval = logging_interval
        self.log_momentum = log_momentum

    def on_train_epoch_start(self, trainer, module):
        opt = trainer.optimizer
        if opt is None:
            return
        name = f"lr-{trainer.optimizer_name}"
        trainer.log_metrics({name: opt.lr}, step=trainer.global_step)


class EarlyStopping(Callback):
    def __init__(self, monitor: str = "loss/total/val", patience: int = 10, mode: str = "min", min_delta: float = 0.0):
        self.monitor, self.patience, self.mode, self.min_delta = monitor, patience, mode, min_delta
        self.wait = 0
        self.best: Optional[float] = None
        self.stopped_epoch = -1

    def on_validation_end(self, trainer, module):
        if trainer.sanity_checking or self.monitor not in trainer.callback_metrics:
            return
        cur = float(trainer.callback_metrics[self.monitor])
        better = self.best is None or (cur < self.best - self.min_delta if self.mode == "min"
                                       else cur > self.best + self.min_delta)
        if better:
            self.best, self.wait = cur, 0
        else:
            self.wait += 1
            if self.wait >= self.patience:
                trainer.should_stop = True
                self.stopped_epoch = trainer.current_epoch

    def state_dict(self):
        return {"wait": self.wait, "best": self.best, "stopped_epoch": self.stopped_epoch}

    def load_state_dict(self, sd):
        self.wait, self.best, self.stopped_epoch = sd.get("wait", 0), sd.get("best"), sd.get("stopped_epoch", -1)


class StepTimer(Callback):
    """Per-epoch throughput: p50/p90 step ms and samples/s from device events (no per-step sync)."""

    def __init__(self):
        self.history: List[Dict[str, float]] = []

    def summarize(self, step_ms: List[float], samples_per_step: int, world: int) -> Dict[str, float]:
        if not step_ms:
            return {}
        s = sorted(step_ms)
        p50 = s[len(s) // 2]
        p90 = s[min(len(s) - 1, int(0.9 * len(s)))]
        rec = {"perf/step_ms_p50": p50, "perf/step_ms_p90": p90,
               "perf/samples_per_s": samples_per_step * world * 1000.0 / max(p50, 1e-9)}
        self.history.append(rec)
        return rec


class DeltaLossReporter(Callback):
    """The thesis' ΔL (`tex/diplomski_rad.tex:1061-1084`): the model's loss minus the loss the
    same decoder gets from the OLS-on-future-window coefficients stored in y channels 2-3 (true α/β on
    synthetic data).  The baseline is parameter-free, so gradients are untouched; this only adds the
    reported values ``delta/{mse,nll,total}/{train,val}`` and ``test/delta_{mse,nll}``.

    The baseline of a split is accumulated once (same fused decoder kernel, same batch size and NLL mode
    as the stage's loader, whole split in order) and cached.  Exact for batch size 1 (the reference
    default) and for ``nll_mode=per_window``; the reference NLL quirk at B > 1 (one Gaussian over the
    batch) depends on the shuffled batch composition, so there it is the in-order baseline."""

    def __init__(self):
        self._cache: Dict[Any, Dict[str, float]] = {}
        self.last: Dict[str, float] = {}

    def _baseline(self, trainer, module, split: str, batch_size: int) -> Dict[str, float]:
        from ..data.loaders import TensorBatchLoader
        from ..ops.losses import decoder_losses

        c_nll, c_mse = module.loss_coefficients
        key = (split, batch_size, c_nll, c_mse, module.nll_mode)
        if key in self._cache:
            return self._cache[key]
        dm = trainer.datamodule
        start, stop = dm.splits[split]
        ld = TensorBatchLoader(dm.dataset, batch_size, shuffle=False, start=start, stop=stop)
        acc = torch.zeros(8, dtype=torch.float64, device=dm.dataset[0].device)
        want_nll = bool(getattr(module, "want_nll", True)) or split == "test"
        with torch.no_grad():
            for x, y, factor, inv_psi in ld:
                B = int(x.shape[0])
                yf = y.flatten(0, 1).float()
                ab = torch.stack([yf[:, 0, 2], yf[:, 0, 3]], -1).contiguous()
                decoder_losses(ab, yf, factor.float(), inv_psi.flatten(0, 1).float(), batch_windows=B,
                               want_nll=want_nll, nll_mode=module.nll_mode, c_nll=c_nll, c_mse=c_mse, acc=acc,
                               with_total=True)
        a = acc.cpu().tolist()
        res = {"mse": a[0] / max(a[1], 1.0), "nll": a[2] / max(a[3], 1.0), "total": a[4] / max(a[5], 1e-30)}
        self._cache[key] = res
        return res

    def _report(self, trainer, module, stage: str, batch_size: int) -> None:
        if trainer.datamodule is None or getattr(trainer.datamodule, "dataset", None) is None:
            return
        base = self._baseline(trainer, module, stage, batch_size)
        out = {}
        for name in ("mse", "nll", "total"):
            tag = f"loss/{name}/{stage}"
            if tag in trainer.callback_metrics:
                out[f"delta/{name}/{stage}"] = float(trainer.callback_metrics[tag]) - base[name]
        if out:
            self.last.update(out)
            trainer.log_metrics(out, step=max(trainer.global_step - 1, 0))

    def on_train_epoch_end(self, trainer, module):
        dm = trainer.datamodule
        self._report(trainer, module, "train", int(dm.hparams["batch_size"]) if dm is not None else 1)

    def on_validation_end(self, trainer, module):
        if not trainer.sanity_checking:
            self._report(trainer, module, "val", 1)

    def on_test_end(self, trainer, module):
        if trainer.datamodule is None or getattr(trainer.datamodule, "dataset", None) is None:
            return
        base = self._baseline(trainer, module, "test", 1)
        acc = module.test_acc.acc.double().cpu().tolist()
        out = {"test/delta_mse": acc[0] / max(acc[1], 1.0) - base["mse"],
               "test/delta_nll": acc[2] / max(acc[3], 1.0) - base["nll"]}
        self.last.update(out)
        trainer.log_metrics(out, step=trainer.global_step)
