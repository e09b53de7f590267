"""Fama-French 25 portfolios (size x book-to-market, daily) loader (reference `src/data.py:62-123`).

Inputs are Kenneth French's two CSVs (``F-F_Research_Data_Factors_daily.csv`` and
``25_Portfolios_5x5_Daily.csv``): a text preamble, a column-header line, then one
``YYYYMMDD,...`` row per day of percent arithmetic returns.  The loader keeps the same
rows as the reference — it drops the preamble, the header and the first
``skip_old_data`` days *and then one more line*, because the reference's
``pandas.read_csv(skiprows=preamble + old, header=0)`` consumes the next line as its
header — and reads ``n_samples - skip_old_data`` days.  Portfolio returns are made
excess (minus RF), days where any portfolio still equals a missing-data marker
(-99.99 / -999) are dropped, and percent returns become percent log-returns
``100·(ln(R + 100) − ln 100)``.  Arithmetic is float32, like the reference.

Returns ``(p25 (25, N), mkt (N,))``.
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Tuple

import numpy as np
import torch
from torch import Tensor

_MISSING = (-99.99, -999.0)


def _read_rows(path: Path, skip_lines: int, nrows: int, ncols: int) -> np.ndarray:
    """Rows ``[skip_lines + 1, skip_lines + 1 + nrows)`` of a CSV as float32 (date column dropped)."""
    import pandas as pd

    df = pd.read_csv(path, header=None, skiprows=skip_lines + 1, nrows=nrows, usecols=range(ncols),
                     dtype=np.float64, skipinitialspace=True)
    return df.to_numpy()[:, 1:].astype(np.float32)


class FamaFrench25Portfolios:
    n_samples = 26129          # days in the files the thesis used
    skip_old_data = 3125       # leading (pre-1939) days dropped
    ff3_filename = "F-F_Research_Data_Factors_daily.csv"
    ff3_skip = 4
    ff3_cols = ["DATE", "Mkt-RF", "SMB", "HML", "RF"]
    p25_filename = "25_Portfolios_5x5_Daily.csv"
    p25_skip = 18
    p25_cols = ["DATE"] + [f"{lo} {hi}" for lo, hi in (
        [("SMALL", "LoBM"), ("ME1", "BM2"), ("ME1", "BM3"), ("ME1", "BM4"), ("SMALL", "HiBM")]
        + [(f"ME{m}", f"BM{b}") for m in (2, 3, 4) for b in range(1, 6)]
        + [("BIG", "LoBM"), ("ME5", "BM2"), ("ME5", "BM3"), ("ME5", "BM4"), ("BIG", "HiBM")])]

    @classmethod
    def load(cls, data_dir) -> Tuple[Tensor, Tensor]:
        d = Path(data_dir)
        f3, f25 = d / cls.ff3_filename, d / cls.p25_filename
        missing = [p.name for p in (f3, f25) if not p.exists()]
        if missing:
            raise FileNotFoundError(
                f"Fama-French raw files {missing} not found in {d}. Download them from Kenneth French's data "
                f"library into that directory (datamodule.raw_dir), or train on datamodule=synthetic.")
        nrows = cls.n_samples - cls.skip_old_data
        ff3 = _read_rows(f3, cls.ff3_skip + cls.skip_old_data, nrows, len(cls.ff3_cols))
        p25 = _read_rows(f25, cls.p25_skip + cls.skip_old_data, nrows, len(cls.p25_cols))
        n = min(len(ff3), len(p25))
        mkt = torch.from_numpy(np.ascontiguousarray(ff3[:n, 0]))                       # Mkt-RF
        rf = torch.from_numpy(np.ascontiguousarray(ff3[:n, 3]))                        # RF
        excess = torch.from_numpy(np.ascontiguousarray(p25[:n].T)) - rf               # (25, n)
        bad = torch.zeros(n, dtype=torch.bool)
        for marker in _MISSING:
            bad |= (excess == torch.tensor(marker, dtype=torch.float32)).any(0)
        excess, mkt = excess[:, ~bad], mkt[~bad]
        ln100 = torch.tensor(math.log(100.0), dtype=torch.float32)
        return 100 * (torch.log(excess + 100) - ln100), 100 * (torch.log(mkt + 100) - ln100)
