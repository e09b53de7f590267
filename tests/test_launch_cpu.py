"""The framework's own multi-process launcher (parallel/launch.py) on the CPU: ``bench.py --gpus N`` and
``train.py trainer.devices=N`` start their N ranks themselves (Lightning's implicit DDP launch,
`/root/reference/train.py:169-180`), report the world that actually ran, and fail as a whole when one rank fails.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parents[1]


def _env(**extra):
    e = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
              "MTA_FAIL_AT_STEP", "MTA_HYDRA_RUN_DIR"):
        e.pop(k, None)
    e.update(extra)
    return e


def test_resolve_devices():
    from masters_thesis_amd.parallel.launch import resolve_devices

    os.environ["HIP_VISIBLE_DEVICES"] = "0,1,2"
    try:
        assert resolve_devices("auto") == 3 and resolve_devices(-1) == 3 and resolve_devices("-1") == 3
        assert resolve_devices(2) == 2 and resolve_devices("4") == 4 and resolve_devices([0, 5]) == 2
        assert resolve_devices("auto", accelerator="cpu") == 1
        with pytest.raises(ValueError):
            resolve_devices(0)
    finally:
        os.environ.pop("HIP_VISIBLE_DEVICES")


@pytest.mark.timeout(300)
def test_bench_launches_its_own_ranks(tmp_path):
    """No torchrun environment: ``--gpus 2`` starts 2 ranks, rank 0 prints the ONE JSON line with n_gpus 2 and
    the process group's world size."""
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--n-samples", "20000"], cwd=tmp_path, env=_env(), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2 and rec["process_group"] == "gloo"
    assert rec["config"]["global_batch"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert "[launch] 2 ranks" in r.stderr


@pytest.mark.timeout(120)
def test_bench_refuses_a_world_other_than_asked(tmp_path):
    """Inside a 1-rank job ``--gpus 2`` must not silently report a 1-rank run as something else."""
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
                        "--n-samples", "20000"], cwd=tmp_path, env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode != 0
    assert "refusing" in r.stderr and not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


@pytest.mark.timeout(300)
def test_train_devices_two_ranks_one_checkpoint_writer(tmp_path):
    """``trainer.devices=2`` (CPU ranks, gloo): both ranks train on their shard, rank 0 alone writes the run's
    .hydra files and checkpoints, and the checkpoint records the world size."""
    r = subprocess.run([sys.executable, str(REPO / "train.py"), "datamodule.n_samples=9000", "trainer.max_epochs=2",
                        "trainer.devices=2", "+trainer.accelerator=cpu"], cwd=tmp_path, env=_env(),
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "[launch] 2 ranks" in r.stderr
    ckdir = tmp_path / "logs/FinancialLstm/synthetic/mse_small_lr0.0001_fast/checkpoints"
    cks = sorted(p.name for p in ckdir.iterdir())
    assert "last.ckpt" in cks and len(cks) == 2, cks
    from masters_thesis_amd.engine.checkpoint import load_checkpoint

    ck = load_checkpoint(ckdir / "last.ckpt", map_location="cpu")
    assert ck["mta"]["world_size"] == 2
    runs = list((tmp_path / "outputs").glob("*/*/.hydra/config.yaml"))
    assert len(runs) == 1, runs


@pytest.mark.timeout(300)
def test_train_devices_rank_failure_fails_the_job(tmp_path):
    """A failing rank ends the whole job with a non-zero status (no rank left waiting in a collective)."""
    r = subprocess.run([sys.executable, str(REPO / "train.py"), "datamodule.n_samples=9000", "trainer.max_epochs=2",
                        "trainer.devices=2", "+trainer.accelerator=cpu"], cwd=tmp_path,
                       env=_env(MTA_FAIL_AT_STEP="3"), capture_output=True, text=True, timeout=280)
    assert r.returncode != 0
    assert "fault injection" in r.stderr or "fault injection" in r.stdout
