"""The framework's own launcher on an MI355X box (parallel/launch.py): ``bench.py --gpus 2`` and ``train.py
trainer.devices=2`` start two ranks themselves.  On a one-GPU box the two ranks share cuda:0 (gloo host group, RCCL
needs a GPU per rank), and the gradient sync is the xGMI/IPC all-reduce kernel inside the captured step -- the code
path an 8-GPU node runs with one rank per GPU.  Reference: Lightning's implicit per-GPU launch,
`/root/reference/train.py:169-180`."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
REPO = Path(__file__).resolve().parents[1]


def _env():
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
              "MTA_FAIL_AT_STEP", "MTA_HYDRA_RUN_DIR"):
        e.pop(k, None)
    return e


@pytest.mark.timeout(300)
def test_bench_gpus2_launches_two_ranks_with_xgmi(tmp_path):
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "40", "--warmup", "5",
                        "--n-samples", "200000"], cwd=tmp_path, env=_env(), capture_output=True, text=True,
                       timeout=280)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    print(json.dumps(rec))
    assert rec["n_gpus"] == 2 and rec["world_size"] == 2, rec
    assert rec["allreduce"] == "xgmi" and rec["allreduce_us"] is not None, rec
    assert rec["visible_devices"] >= 1 and rec["value"] > 0


@pytest.mark.timeout(400)
def test_train_devices2_one_checkpoint_from_rank0(tmp_path):
    r = subprocess.run([sys.executable, str(REPO / "train.py"), "datamodule.n_samples=50000", "seed=0",
                        "trainer.max_epochs=2", "trainer.devices=2", "trainer.enable_progress_bar=false"],
                       cwd=tmp_path, env=_env(), capture_output=True, text=True, timeout=380)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-4000:]
    assert "[launch] 2 ranks" in r.stderr
    ckdir = tmp_path / "logs/FinancialLstm/synthetic/mse_small_lr0.0001_fast/checkpoints"
    cks = sorted(p.name for p in ckdir.iterdir())
    assert "last.ckpt" in cks and len(cks) == 2, cks
    from masters_thesis_amd.engine.checkpoint import load_checkpoint

    ck = load_checkpoint(ckdir / "last.ckpt", map_location="cpu")
    assert ck["mta"]["world_size"] == 2 and ck["epoch"] == 1
    assert "Test MAE" in r.stdout
