"""Serialize / launch-blocking debug mode plumbing (masters_thesis_amd/utils/debug.py; SURVEY §5 race detection)."""
import os

from masters_thesis_amd.utils.debug import SERIALIZE_ENV


def _clear(monkeypatch):
    for k in (*SERIALIZE_ENV, "MTA_DEBUG_SERIALIZE"):
        monkeypatch.delenv(k, raising=False)


def test_trainer_flag_exports_serialize_env_and_disables_graphs(monkeypatch):
    from masters_thesis_amd.engine import Trainer

    _clear(monkeypatch)
    tr = Trainer(enable_progress_bar=False, enable_model_summary=False, debug_serialize=True, steps_per_graph=8)
    assert tr.debug_serialize
    for k, v in SERIALIZE_ENV.items():
        assert os.environ[k] == v
    assert os.environ["AMD_SERIALIZE_KERNEL"] == "3" and os.environ["HIP_LAUNCH_BLOCKING"] == "1"
    assert not tr.use_hip_graphs and tr.steps_per_graph == 1


def test_env_switch_and_default_off(monkeypatch):
    from masters_thesis_amd.engine import Trainer

    _clear(monkeypatch)
    tr = Trainer(enable_progress_bar=False, enable_model_summary=False)
    assert not tr.debug_serialize and "AMD_SERIALIZE_KERNEL" not in os.environ and tr.use_hip_graphs
    monkeypatch.setenv("MTA_DEBUG_SERIALIZE", "1")
    tr = Trainer(enable_progress_bar=False, enable_model_summary=False)
    assert tr.debug_serialize and os.environ["AMD_SERIALIZE_COPY"] == "3" and not tr.use_hip_graphs


def test_train_py_passes_config_key(monkeypatch):
    import train
    from masters_thesis_amd.config import compose
    from pathlib import Path

    _clear(monkeypatch)
    root = Path(train.__file__).resolve().parent
    cfg, _, _ = compose(root / "configs", "config", ["+trainer.debug_serialize=true"])
    tr = train.build_trainer(cfg, None, [])
    assert tr.debug_serialize and not tr.use_hip_graphs
