"""Training engine (Lightning-compatible loops, callbacks, checkpoints, HIP-graph step capture)."""
from .callbacks import Callback, DeltaLossReporter, EarlyStopping, LearningRateMonitor, ModelCheckpoint, StepTimer
from .module import LightningModule
from .trainer import Trainer

__all__ = ["Callback", "DeltaLossReporter", "EarlyStopping", "LearningRateMonitor", "ModelCheckpoint", "StepTimer", "LightningModule",
           "Trainer"]
