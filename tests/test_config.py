"""Config composer: golden behaviour of every override form used by the reference
(`train.py:75-93`, `sweeps/*.sh`, `configs/config.yaml`)."""
from pathlib import Path

import pytest

from masters_thesis_amd.config import (ConfigCompositionError, OmegaConf, compose, expand_sweep, parse_override)

CFG = Path(__file__).resolve().parents[1] / "configs"


def test_defaults_compose_like_reference():
    cfg, hy, choices = compose(CFG, "config", [])
    assert choices == {"datamodule": "synthetic", "model": "small", "loss": "mse", "trainer": "fast"}
    assert cfg.model.input_size == 3  # custom resolver input_size_from_interaction
    assert cfg.logger.name == "FinancialLstm/synthetic"
    assert cfg.logger.version == "mse_small_lr0.0001_fast"
    assert cfg.trainer.precision == "32-true"
    assert "check_val_every_n_epoch" not in cfg.trainer
    assert hy.launcher["_target_"] == "joblib" and hy.launcher.n_jobs == 1
    assert "hydra" not in cfg


def test_group_and_value_overrides():
    cfg, _, _ = compose(CFG, "config", ["loss=combined", "loss.mse_weight=0.7", "model=large",
                                        "model.learning_rate=0.00001", "datamodule=real", "trainer=slow"])
    assert cfg.loss.module_class == "FinancialLstmCombined" and cfg.loss.mse_weight == 0.7
    assert cfg.model.num_layers == 8 and cfg.model.dropout == 0.3
    assert cfg.logger.version == "combined_large_lr1e-05_slow"
    assert cfg.logger.name == "FinancialLstm/real"
    assert cfg.datamodule.stride == 5
    assert cfg.trainer.check_val_every_n_epoch == 4


def test_interaction_only_false_changes_input_size():
    cfg, _, _ = compose(CFG, "config", ["datamodule.interaction_only=false"])
    assert cfg.model.input_size == 5


def test_add_delete_force_add():
    cfg, _, _ = compose(CFG, "config", ["+trainer.use_hip_graphs=false", "~checkpoint", "++seed=7"])
    assert cfg.trainer.use_hip_graphs is False
    assert "checkpoint" not in cfg
    assert cfg.seed == 7
    with pytest.raises(KeyError):
        compose(CFG, "config", ["trainer.not_a_key=1"])
    with pytest.raises(ConfigCompositionError):
        compose(CFG, "config", ["+trainer.max_epochs=3"])


def test_unknown_group_option_and_sweep_without_multirun():
    with pytest.raises(ConfigCompositionError):
        compose(CFG, "config", ["model=huge"])
    with pytest.raises(ConfigCompositionError):
        compose(CFG, "config", ["loss=mse,nll"])


def test_sweep_expansion_matches_reference_scripts():
    syn = [parse_override(x) for x in ["datamodule=synthetic", "model=small,medium,large", "loss=mse,nll,combined",
                                       "trainer=fast,slow"]]
    jobs = expand_sweep(syn)
    assert len(jobs) == 18
    assert [o.text() for o in jobs[0]] == ["datamodule=synthetic", "model=small", "loss=mse", "trainer=fast"]
    assert [o.text() for o in jobs[-1]] == ["datamodule=synthetic", "model=large", "loss=combined", "trainer=slow"]
    ex = [parse_override(x) for x in ["datamodule=real", "model=large", "model.learning_rate=0.001,0.0001,0.00001",
                                      "trainer.max_epochs=100,200"]]
    jobs = expand_sweep(ex)
    assert len(jobs) == 6
    versions = set()
    for j in jobs:
        cfg, _, _ = compose(CFG, "config", j)
        versions.add(cfg.logger.version)
    # max_epochs is not part of logger.version: 3 distinct version dirs for 6 jobs
    assert versions == {"mse_large_lr0.001_fast", "mse_large_lr0.0001_fast", "mse_large_lr1e-05_fast"}


def test_range_sweep_and_parse_scalars():
    o = parse_override("x=range(1,4)")
    assert o.is_sweep and o.value == [1, 2, 3]
    assert parse_override("a=null").value is None
    assert parse_override("a=1e-05").value == 1e-05
    assert parse_override("a='1,2'").value == "1,2"
    assert parse_override("a=[1,2]").value == [1, 2]


def test_to_container_resolves_and_yaml_roundtrip(tmp_path):
    cfg, _, _ = compose(CFG, "config", ["loss=nll"])
    d = OmegaConf.to_container(cfg, resolve=True)
    assert d["logger"]["version"] == "nll_small_lr0.0001_fast"
    assert d["model"]["input_size"] == 3
    OmegaConf.save(cfg, tmp_path / "c.yaml")
    back = OmegaConf.load(tmp_path / "c.yaml")
    assert back.loss.name == "nll"


def test_launcher_override_and_hydra_node():
    _, hy, _ = compose(CFG, "config", ["hydra/launcher=gpu_pool", "hydra.launcher.jobs_per_device=3"])
    assert hy.launcher["_target_"] == "gpu_pool" and hy.launcher.jobs_per_device == 3
    assert str(hy.sweep.subdir) == "0"


def test_jobs_per_device_capped_at_measured_optimum():
    """Trial packing beyond 4 per GPU measured slower in aggregate (profiles/r4_pack_sweep.jsonl): capped unless
    max_jobs_per_device is raised."""
    from masters_thesis_amd.config.app import MAX_JOBS_PER_DEVICE, jobs_per_device

    _, hy, _ = compose(CFG, "config", ["hydra/launcher=gpu_pool", "hydra.launcher.jobs_per_device=8"])
    assert hy.launcher.max_jobs_per_device == MAX_JOBS_PER_DEVICE == 4
    assert jobs_per_device(hy.launcher) == 4
    assert jobs_per_device({"jobs_per_device": 3}) == 3
    assert jobs_per_device({"jobs_per_device": 8, "max_jobs_per_device": 8}) == 8
