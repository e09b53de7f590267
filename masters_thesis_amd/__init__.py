"""masters_thesis_amd — an MI355X-native (gfx950) trainer for latent-factor return models.

Capabilities of MarkoMiljkovic45/masters-thesis (LSTM alpha/beta encoder trained with
MSE / Woodbury-NLL / combined decoders on synthetic or Fama-French data, Hydra configs,
sweeps, Lightning-style checkpoints and TensorBoard logs), rebuilt on PyTorch-ROCm +
hand-written CDNA4 HIP kernels + RCCL over xGMI.
"""
__version__ = "0.1.0"

from .data import FinancialLstmDataModule, FamaFrench25Portfolios, SyntheticLogReturns  # noqa: E402
from .models import FinancialLstm, FinancialLstmCombined, FinancialLstmMse, FinancialLstmNll  # noqa: E402

__all__ = ["SyntheticLogReturns", "FamaFrench25Portfolios", "FinancialLstmDataModule", "FinancialLstm",
           "FinancialLstmMse", "FinancialLstmNll", "FinancialLstmCombined"]
