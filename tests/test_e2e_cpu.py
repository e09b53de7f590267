"""End-to-end CPU runs of the CLI (BASELINE.json config 1): train -> checkpoint -> test,
multirun, resume / init_from, fault injection, TensorBoard event files."""
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch

REPO = Path(__file__).resolve().parents[1]
TINY = ["datamodule.n_samples=9000", "datamodule.n_stocks=100"]


def _run(args, cwd, env=None, ok=True, timeout=600):
    e = dict(os.environ)
    e.pop("MTA_FAIL_AT_STEP", None)
    e.update(env or {})
    e["CUDA_VISIBLE_DEVICES"] = ""
    e["HIP_VISIBLE_DEVICES"] = ""
    # a few OpenMP threads per training process: pytest -n workers x launcher children x torch's default of one
    # spinning thread per core oversubscribe the host by an order of magnitude
    e.setdefault("OMP_NUM_THREADS", "2")
    r = subprocess.run([sys.executable, *args], cwd=cwd, env=e, capture_output=True, text=True, timeout=timeout)
    if ok and r.returncode != 0:
        raise AssertionError(f"{args} failed ({r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}")
    return r


@pytest.fixture(scope="module")
def trained(tmp_path_factory):
    d = tmp_path_factory.mktemp("e2e")
    r = _run([str(REPO / "train.py"), *TINY, "trainer.max_epochs=2", "loss=combined"], d)
    vdir = d / "logs/FinancialLstm/synthetic/combined_small_lr0.0001_fast"
    return d, vdir, r.stdout


def test_train_writes_reference_layout(trained):
    d, vdir, out = trained
    ck = sorted((vdir / "checkpoints").glob("*.ckpt"))
    names = [p.name for p in ck]
    assert "last.ckpt" in names and any(n.startswith("best_epoch=") and "_val=" in n for n in names)
    sd = torch.load(vdir / "checkpoints/last.ckpt", weights_only=True, map_location="cpu")
    for key in ("epoch", "global_step", "pytorch-lightning_version", "state_dict", "loops", "callbacks",
                "optimizer_states", "lr_schedulers", "hparams_name", "hyper_parameters"):
        assert key in sd, key
    assert set(sd["state_dict"]) == {
        *(f"lstm.{w}_l{k}" for k in range(2) for w in ("weight_ih", "weight_hh", "bias_ih", "bias_hh")),
        "alpha_head.weight", "alpha_head.bias", "beta_head.weight", "beta_head.bias"}
    assert sd["hyper_parameters"]["mse_weight"] == 100
    assert "Test MAE" in out and "Best validation loss" in out
    assert (d / "outputs").exists() and list((d / "outputs").glob("*/*/.hydra/config.yaml"))


def test_tfevents_have_reference_tags(trained):
    from masters_thesis_amd.utils.tfevents import read_scalars, read_tags

    _, vdir, _ = trained
    ev = sorted(vdir.glob("events.out.tfevents.*"))
    assert ev
    sc = read_scalars(ev[0])
    for tag in ("loss/mse/train", "loss/nll/train", "loss/total/train", "loss/mse/val", "loss/nll/val",
                "loss/total/val", "lr-Adam"):
        assert tag in sc, (tag, sorted(sc))
    assert len(sc["loss/total/val"]) == 2
    tags = read_tags(ev[0])
    assert any("hparams" in t or t.startswith("_hparams_") for t in tags) or "test/mae" in sc


def test_test_py_on_checkpoint_writes_figures(trained):
    from masters_thesis_amd.utils.tfevents import read_tags

    d, vdir, _ = trained
    _run([str(REPO / "test.py"), *TINY, "loss=combined",
          "checkpoint=logs/FinancialLstm/synthetic/combined_small_lr0.0001_fast/checkpoints/last.ckpt"], d)
    tags = set()
    for ev in vdir.rglob("events.out.tfevents.*"):
        tags |= set(read_tags(ev))
    for t in ("scatter/recon_residuals", "scatter/alphas", "scatter/betas", "hist/alphas", "hist/betas"):
        assert t in tags, (t, sorted(tags))


def test_resume_and_init_from(trained):
    d, vdir, _ = trained
    last = vdir / "checkpoints/last.ckpt"
    r = _run([str(REPO / "train.py"), *TINY, "trainer.max_epochs=3", "loss=combined", f"resume={last}",
              "logger.version=resumed"], d)
    sd = torch.load(d / "logs/FinancialLstm/synthetic/resumed/checkpoints/last.ckpt", weights_only=True)
    assert sd["epoch"] == 2, sd["epoch"]
    r = _run([str(REPO / "train.py"), *TINY, "trainer.max_epochs=1", "loss=mse", f"init_from={last}",
              "logger.version=warm"], d)
    assert "Initialised weights from" in r.stdout


def test_fault_injection_then_resume(tmp_path):
    r = _run([str(REPO / "train.py"), *TINY, "trainer.max_epochs=2", "logger.version=faulty"], tmp_path,
             env={"MTA_FAIL_AT_STEP": "90"}, ok=False)
    assert r.returncode != 0 and "fault injection" in (r.stdout + r.stderr)
    ck = tmp_path / "logs/FinancialLstm/synthetic/faulty/checkpoints/last.ckpt"
    assert ck.exists()  # epoch 0 finished (70 train batches) before the fault at step 90
    _run([str(REPO / "train.py"), *TINY, "trainer.max_epochs=2", "logger.version=faulty", f"resume={ck}"], tmp_path)


def test_multirun_expands_and_runs_each_job(tmp_path):
    r = _run([str(REPO / "train.py"), "-m", *TINY, "trainer.max_epochs=1", "model.learning_rate=0.001,0.0001"],
             tmp_path)
    runs = sorted((tmp_path / "multirun").glob("*/*/[0-9]*"))
    assert len(runs) == 2, runs
    for v in ("mse_small_lr0.001_fast", "mse_small_lr0.0001_fast"):
        assert (tmp_path / "logs/FinancialLstm/synthetic" / v / "checkpoints/last.ckpt").exists()


def test_report_delta_and_best_ckpt(tmp_path):
    """SURVEY Q10 (ΔL vs the OLS-on-future-window baseline, `tex/diplomski_rad.tex:1061-1084`) and Q9
    (``test_ckpt=best`` tests the best-validation weights, `train.py:198` tests the last ones)."""
    from masters_thesis_amd.utils.tfevents import read_scalars

    r = _run([str(REPO / "train.py"), *TINY, "trainer.max_epochs=2", "loss=combined", "report_delta=true",
              "test_ckpt=best", "logger.version=delta"], tmp_path)
    assert "Testing best weights" in r.stdout and "Test ΔNLL" in r.stdout
    vdir = tmp_path / "logs/FinancialLstm/synthetic/delta"
    sc = read_scalars(sorted(vdir.glob("events.out.tfevents.*"))[0])
    for tag in ("delta/total/train", "delta/mse/val", "delta/nll/val", "delta/total/val", "test/delta_mse",
                "test/delta_nll"):
        assert tag in sc, (tag, sorted(sc))
    # ΔL = L(model) - L(OLS baseline): the implied baseline is non-negative and the same every epoch
    base = [lv - dv for (_, lv), (_, dv) in zip(sc["loss/mse/val"], sc["delta/mse/val"])]
    assert len(base) == 2 and base[0] >= 0 and abs(base[0] - base[1]) <= 1e-5 * max(base[0], 1e-12), base
    bad = _run([str(REPO / "train.py"), *TINY, "trainer.max_epochs=1", "test_ckpt=worst", "logger.version=bad"],
               tmp_path, ok=False)
    assert bad.returncode != 0 and "test_ckpt" in (bad.stdout + bad.stderr)


def test_launcher_retries_failed_trial_with_auto_resume(tmp_path):
    """SURVEY §5 failure handling: a trial that dies (fault injection on its first attempt only) is re-queued by
    the child-process launcher with resume=auto and finishes from its own last.ckpt."""
    r = _run([str(REPO / "train.py"), "-m", *TINY, "trainer.max_epochs=2", "model.learning_rate=0.001,0.0001",
              "hydra/launcher=joblib", "hydra.launcher.n_jobs=2", "hydra.launcher.max_retries=1"], tmp_path,
             env={"MTA_FAIL_AT_STEP": "90", "MTA_FAIL_ATTEMPTS": "1"})
    assert r.stdout.count("retry 1/1 with resume=auto") == 2, r.stdout
    outs = sorted((tmp_path / "multirun").glob("*/*/job*.out"))
    assert len(outs) == 2
    for o in outs:
        text = o.read_text()
        assert "fault injection" in text and "resuming from" in text and "Test MAE" in text
    for v in ("mse_small_lr0.001_fast", "mse_small_lr0.0001_fast"):
        ck = torch.load(tmp_path / "logs/FinancialLstm/synthetic" / v / "checkpoints/last.ckpt", weights_only=True)
        assert ck["epoch"] == 1


def test_gpu_pool_launcher_pins_one_device_per_slot(tmp_path):
    """hydra/launcher=gpu_pool: every trial is a child process with its own HIP_VISIBLE_DEVICES slot (two fake
    devices here; on CPU the children train on the CPU), results land in per-job run dirs."""
    r = _run([str(REPO / "train.py"), "-m", *TINY, "trainer.max_epochs=1", "model.learning_rate=0.001,0.0001",
              "hydra/launcher=gpu_pool", "hydra.launcher.devices=2", "hydra.launcher.jobs_per_device=1"], tmp_path)
    assert "[launcher:gpu_pool] job #0 (attempt 0) on slot 0" in r.stdout, r.stdout
    assert "[launcher:gpu_pool] job #1 (attempt 0) on slot 1" in r.stdout, r.stdout
    outs = sorted((tmp_path / "multirun").glob("*/*/job*.out"))
    assert len(outs) == 2 and all("Test MAE" in o.read_text() for o in outs)
