"""Training entry point (same CLI/config contract as the reference `train.py`).

    python train.py                                   # defaults: synthetic, small, mse, fast
    python train.py loss=nll
    python train.py loss=combined loss.mse_weight=0.7
    python train.py datamodule=real model=large loss=combined trainer=slow
    python train.py -m loss=mse,nll,combined model=small,medium,large
    python train.py -m loss=combined loss.mse_weight=0.3,0.5,0.7
    python train.py trainer.devices=8                 # DDP, one process per MI355X (RCCL/xGMI), own launcher
                                                      # (trainer.devices=auto, the default: every visible GPU)
    torchrun --nproc-per-node 8 train.py ...          # the same under an external launcher

MI355X additions (all optional): ``resume=<ckpt>|auto`` (full state; ``auto`` = this run's own
last.ckpt if present, used by the launcher's retries), ``init_from=<ckpt>``
(weights only: the thesis' synthetic->real warm-up), ``seed=<int>``,
``+trainer.use_hip_graphs=false``, ``+trainer.matmul_precision=highest|high|medium``,
``trainer.precision=bf16-mixed``, ``hydra/launcher=gpu_pool`` (one trial per GPU),
``test_ckpt=best`` (test the best-validation weights instead of the last ones),
``report_delta=true`` (log ΔL = model loss minus the OLS-on-future-window loss).
"""
from __future__ import annotations

import os
import time
from pathlib import Path

import torch

from masters_thesis_amd.config import OmegaConf, main as config_main, register_default_resolvers
from masters_thesis_amd.data import FinancialLstmDataModule
from masters_thesis_amd.engine import DeltaLossReporter, EarlyStopping, LearningRateMonitor, ModelCheckpoint, Trainer
from masters_thesis_amd.engine.checkpoint import load_checkpoint
from masters_thesis_amd.models import get_model_class, model_params_from_config
from masters_thesis_amd.utils.logger import TensorBoardLogger

# reference `train.py:13` (allows reduced-precision fp32 matmuls in plain PyTorch ops)
torch.set_float32_matmul_precision("medium")
register_default_resolvers()


def build_trainer(cfg, logger, callbacks):
    t = cfg.trainer
    kw = dict(
        max_epochs=t.max_epochs,
        gradient_clip_val=t.gradient_clip_val,
        precision=t.precision,
        enable_progress_bar=t.enable_progress_bar,
        enable_model_summary=t.enable_model_summary,
        logger=logger,
        callbacks=callbacks,
    )
    if "check_val_every_n_epoch" in t:
        kw["check_val_every_n_epoch"] = t.check_val_every_n_epoch
    for k in ("use_hip_graphs", "matmul_precision", "limit_train_batches", "limit_val_batches",
              "limit_test_batches", "accelerator", "num_sanity_val_steps", "max_steps", "graph_warmup_steps",
              "steps_per_graph", "deterministic", "log_every_n_steps", "profiler", "profile_steps",
              "debug_serialize", "devices"):
        if k in t:
            kw[k] = t[k]
    return Trainer(**kw)


@config_main(version_base=None, config_path="configs", config_name="config")
def main(cfg):
    print("\n" + "=" * 70)
    print("EXPERIMENT CONFIGURATION")
    print("=" * 70)
    print(f"Datamodule: {cfg.datamodule.name}")
    print(f"Model: {cfg.model.name} (hidden={cfg.model.hidden_size}, layers={cfg.model.num_layers})")
    print(f"Loss: {cfg.loss.name} (class={cfg.loss.module_class})")
    if cfg.loss.name == "combined":
        print(f"  └─ MSE Weight: {cfg.loss.mse_weight}")
    print(f"Trainer: {cfg.trainer.name} (epochs={cfg.trainer.max_epochs})")
    print(f"Learning Rate: {cfg.model.learning_rate}")
    print(f"Logger: {cfg.logger.name}/{cfg.logger.version}")
    print("=" * 70 + "\n")

    if cfg.get("seed") is not None:
        torch.manual_seed(int(cfg.seed))

    # ==================== DataModule ====================
    dm = FinancialLstmDataModule.from_config(cfg.datamodule)

    # ==================== Model ====================
    ModelClass = get_model_class(cfg.loss.module_class, cfg.model.get("arch", "lstm"))
    model = ModelClass(**model_params_from_config(cfg))
    if cfg.get("init_from"):
        ck = load_checkpoint(cfg.init_from, map_location="cpu")
        model.load_state_dict(ck["state_dict"])
        print(f"Initialised weights from {cfg.init_from}")
    model.compile()
    print(model)
    print(f"\nUsing Lightning Module: {ModelClass.__name__}\n")

    # ==================== Logger / callbacks ====================
    tb_logger = TensorBoardLogger(save_dir=cfg.logger.save_dir, name=cfg.logger.name, version=cfg.logger.version,
                                  default_hp_metric=cfg.logger.default_hp_metric,
                                  rank=int(os.environ.get("RANK", "0")))
    checkpoint_dir = Path(cfg.logger.save_dir) / cfg.logger.name / cfg.logger.version / "checkpoints"
    callbacks = [
        ModelCheckpoint(dirpath=str(checkpoint_dir), filename="best_epoch={epoch:02d}_val={loss/total/val:.4f}",
                        monitor="loss/total/val", mode="min", save_last=True, auto_insert_metric_name=False),
        LearningRateMonitor(logging_interval="epoch", log_momentum=False),
    ]
    delta = None
    if cfg.get("report_delta"):
        delta = DeltaLossReporter()
        callbacks.append(delta)
    if cfg.trainer.get("early_stopping_patience"):
        callbacks.append(EarlyStopping(monitor="loss/total/val", patience=int(cfg.trainer.early_stopping_patience)))

    trainer = build_trainer(cfg, tb_logger, callbacks)

    print("\n" + "=" * 50)
    print("Starting Training...")
    print("=" * 50 + "\n")
    resume = cfg.get("resume")
    if resume == "auto":
        # launcher retries (max_retries): continue from this run's own last checkpoint when there is one
        last = checkpoint_dir / "last.ckpt"
        resume = str(last) if last.exists() else None
        print(f"resume=auto: {'resuming from ' + resume if resume else 'no checkpoint yet, starting fresh'}")
    step0 = trainer.global_step
    t_fit = time.perf_counter()
    trainer.fit(model, datamodule=dm, ckpt_path=resume)
    t_fit = time.perf_counter() - t_fit
    # one machine-readable line per trial (scripts/gpu_sweep_throughput.sh sums them over a sweep)
    n_windows = (trainer.global_step - step0) * int(cfg.datamodule.batch_size)
    print(f"[throughput] train_windows={n_windows} fit_s={t_fit:.3f} windows_per_s={n_windows / max(t_fit, 1e-9):.1f}",
          flush=True)

    ckpt_cb = trainer.checkpoint_callback
    best = ckpt_cb.best_model_score
    print("\n" + "=" * 50)
    print("Training Complete!")
    print("=" * 50)
    print(f"Best model path: {ckpt_cb.best_model_path}")
    print(f"Best validation loss: {float(best) if best is not None else float('nan'):.6f}")
    print("=" * 50 + "\n")

    # ==================== Test (last weights like the reference, or the best ones: SURVEY Q9) ==========
    test_ckpt = str(cfg.get("test_ckpt") or "last")
    if test_ckpt not in ("best", "last"):
        raise ValueError(f"test_ckpt must be 'best' or 'last', got {test_ckpt!r}")
    if test_ckpt == "best" and ckpt_cb.best_model_path:
        model.load_state_dict(load_checkpoint(ckpt_cb.best_model_path, map_location="cpu")["state_dict"])
        print(f"Testing best weights: {ckpt_cb.best_model_path}")
    trainer.test(model, datamodule=dm)

    config_dict = OmegaConf.to_container(cfg, resolve=True)
    config_dict.pop("logger", None)
    tb_logger.log_hyperparams(
        params=config_dict,
        metrics={
            "test/mae": model.test_results["test_loss"]["mae"],
            "test/nll": model.test_results["test_loss"]["nll"],
            "test/best_val_loss": float(best) if best is not None else float("nan"),
            **({k: v for k, v in delta.last.items() if k.startswith("test/")} if delta is not None else {}),
        },
    )
    tb_logger.close()

    print("\n" + "=" * 50)
    print("FINAL TEST RESULTS")
    print("=" * 50)
    print(f"Test MAE: {model.test_results['test_loss']['mae']:.6f}")
    print(f"Test NLL: {model.test_results['test_loss']['nll']:.6f}")
    if delta is not None:
        print(f"Test ΔMSE: {delta.last.get('test/delta_mse', float('nan')):.6f}")
        print(f"Test ΔNLL: {delta.last.get('test/delta_nll', float('nan')):.6f}")
    print("=" * 50 + "\n")
    return float(best) if best is not None else None


if __name__ == "__main__":
    main()
