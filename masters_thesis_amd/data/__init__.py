"""Data: synthetic DGP, Fama-French 25 loader, windowing + OLS targets, data module and loaders
(reference `src/data.py`, `src/common.py`)."""
from .common import (add_quadratic_features, gaussian_nll_dense, inverse_returns_covariance, lookback_target_split,
                     ols, ols_features, woodbury_nll_closed_form)
from .datamodule import FinancialLstmDataModule, build_windows
from .dgp import SyntheticLogReturns
from .famafrench import FamaFrench25Portfolios
from .loaders import TensorBatchLoader
from .prefetch import StreamingLoader

__all__ = ["SyntheticLogReturns", "FamaFrench25Portfolios", "FinancialLstmDataModule", "TensorBatchLoader",
           "StreamingLoader", "build_windows", "ols", "ols_features", "lookback_target_split",
           "add_quadratic_features", "inverse_returns_covariance", "gaussian_nll_dense", "woodbury_nll_closed_form"]
