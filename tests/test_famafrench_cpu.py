"""Fama-French 25 loader (`src/data.py:62-123`) and datamodule=real end to end, on synthetic CSVs.

No Kenneth French data ships with the reference and there is no network, so the raw files are
generated here in the library's layout (preamble lines, a column-header line, YYYYMMDD rows of
percent returns); the expected tensors come from an independent numpy reading of the same rows.
"""
import math
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

from masters_thesis_amd.data.famafrench import FamaFrench25Portfolios as FF

REPO = Path(__file__).resolve().parents[1]
N_ROWS = FF.n_samples + 40  # data rows in the files (more than the loader reads)


def _write_raw(d: Path, seed: int = 0):
    rng = np.random.default_rng(seed)
    dates = 19260701 + np.arange(N_ROWS)
    mkt = np.round(rng.normal(0.05, 1.0, N_ROWS), 2)
    rf = np.round(rng.uniform(0.0, 0.03, N_ROWS), 3)
    p25 = np.round(rng.normal(0.05, 1.2, (N_ROWS, 25)), 2)
    first = FF.skip_old_data  # first data row the loader keeps (see _expected)
    # missing markers: dropped only where P - RF still equals the marker (RF == 0), like the reference
    rf[first + 10] = 0.0
    p25[first + 10, 3] = -99.99
    rf[first + 20] = 0.0
    p25[first + 20, 7] = -999
    ff3_lines = ["This file was created synthetically", "", "", ""]
    ff3_lines.append(",Mkt-RF,SMB,HML,RF")
    for i in range(N_ROWS):
        ff3_lines.append(f"{dates[i]},{mkt[i]:.2f},0.10,-0.10,{rf[i]:.3f}")
    (d / FF.ff3_filename).write_text("\n".join(ff3_lines) + "\n")
    p_lines = [f"preamble {i}" for i in range(FF.p25_skip)]
    p_lines.append("," + ",".join(FF.p25_cols[1:]))
    for i in range(N_ROWS):
        p_lines.append(f"{dates[i]}," + ",".join(f"{v:.2f}" for v in p25[i]))
    (d / FF.p25_filename).write_text("\n".join(p_lines) + "\n")
    return mkt, rf, p25


def _expected(mkt, rf, p25):
    # skiprows = preamble + old rows; the next line is consumed as the header (replaced by `names`)
    start = FF.skip_old_data
    rows = slice(start, start + FF.n_samples - FF.skip_old_data)
    m = mkt[rows].astype(np.float32)
    r = rf[rows].astype(np.float32)
    P = p25[rows].astype(np.float32).T - r
    keep = ~((P == np.float32(-99.99)).any(0) | (P == np.float32(-999)).any(0))
    P, m = P[:, keep], m[keep]
    return (100 * (np.log(P + 100) - math.log(100))).astype(np.float32), \
        (100 * (np.log(m + 100) - math.log(100))).astype(np.float32), keep


def test_ff25_load_matches_numpy(tmp_path):
    raw = _write_raw(tmp_path)
    p25, mkt = FF.load(tmp_path)
    ep, em, keep = _expected(*raw)
    assert p25.shape == (25, keep.sum()) and mkt.shape == (keep.sum(),)
    assert keep.sum() == FF.n_samples - FF.skip_old_data - 2
    np.testing.assert_allclose(p25.numpy(), ep, rtol=1e-5, atol=1e-4)  # float32 log
    np.testing.assert_allclose(mkt.numpy(), em, rtol=1e-5, atol=1e-4)


def test_ff25_missing_files_raise(tmp_path):
    with pytest.raises(FileNotFoundError, match="datamodule=synthetic"):
        FF.load(tmp_path)


def test_train_on_real_datamodule(tmp_path):
    raw_dir = tmp_path / "raw"
    raw_dir.mkdir()
    _write_raw(raw_dir)
    args = [sys.executable, str(REPO / "train.py"), "datamodule=real", f"datamodule.raw_dir={raw_dir}",
            f"datamodule.data_dir={tmp_path / 'real'}", "trainer.max_epochs=1",
            "+trainer.limit_train_batches=40", "+trainer.limit_val_batches=10", "+trainer.limit_test_batches=10"]
    env = {"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": "", "PATH": "/usr/bin:/bin", "OMP_NUM_THREADS": "2"}
    r = subprocess.run(args, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    stocks = torch.load(tmp_path / "real/stocks.pt", weights_only=True)
    assert stocks.shape[0] == 25
    ds = tmp_path / "real/datasets"
    assert (ds / "hparams_hash.txt").exists()
    vdir = tmp_path / "logs/FinancialLstm/real/mse_small_lr0.0001_fast/checkpoints"
    assert (vdir / "last.ckpt").exists()
