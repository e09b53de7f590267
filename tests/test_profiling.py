"""Tracing hooks (SURVEY.md §5 "Tracing / profiling"): per-phase device timers and the torch.profiler hook."""
import json
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parents[1]


def _fit(tmp_path, device, **trainer_kw):
    from masters_thesis_amd.config import compose
    from masters_thesis_amd.data import FinancialLstmDataModule
    from masters_thesis_amd.engine import Trainer
    from masters_thesis_amd.models import get_model_class, model_params_from_config

    cfg, _, _ = compose(REPO / "configs", "config", ["datamodule.n_samples=4000", "datamodule.n_stocks=100",
                                                     f"datamodule.data_dir={tmp_path}"])
    dm = FinancialLstmDataModule.from_config(cfg.datamodule, cache=False, device=torch.device(device))
    torch.manual_seed(0)
    model = get_model_class(cfg.loss.module_class, "lstm")(**model_params_from_config(cfg))
    tr = Trainer(max_epochs=1, gradient_clip_val=5.0, enable_progress_bar=False, enable_model_summary=False,
                 logger=None, callbacks=[], num_sanity_val_steps=0, limit_train_batches=12, limit_val_batches=2,
                 accelerator="cpu" if device == "cpu" else "auto", default_root_dir=str(tmp_path), **trainer_kw)
    tr.fit(model, datamodule=dm)
    return tr


def test_phase_timers_cpu(tmp_path):
    tr = _fit(tmp_path, "cpu", profiler="phases")
    ph = {k: v for k, v in tr.perf.items() if k.startswith("perf/phase/")}
    for name in ("gather", "fwd", "bwd", "optim"):
        assert f"perf/phase/{name}_ms_p50" in ph, ph
        assert ph[f"perf/phase/{name}_ms_p50"] >= 0.0
    assert tr.perf["perf/step_ms_p50"] == pytest.approx(sum(ph.values()))


def test_torch_profiler_trace_cpu(tmp_path):
    tr = _fit(tmp_path, "cpu", profiler="torch", profile_steps=3)
    path = Path(tr.torch_trace_path)
    assert path.exists()
    trace = json.loads(path.read_text())
    assert trace.get("traceEvents"), "empty trace"


def test_profiler_name_checked():
    from masters_thesis_amd.engine import Trainer

    with pytest.raises(ValueError):
        Trainer(profiler="nsys")


@pytest.mark.gpu
def test_phase_timers_gpu(tmp_path):
    tr = _fit(tmp_path, "cuda", profiler="phases")
    ph = {k: v for k, v in tr.perf.items() if k.startswith("perf/phase/")}
    # fused training step: fwd (pipelined LSTM), loss (decoder), bwd (pipelined BPTT + wgrad), optim (clip+Adam)
    for name in ("gather", "fwd", "loss", "bwd", "optim"):
        assert ph.get(f"perf/phase/{name}_ms_p50", 0.0) > 0.0, ph
