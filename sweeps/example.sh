#!/bin/bash
# Learning-rate x epochs grid on the real (FF25) data with the large LSTM: 3 x 2 = 6 jobs.
# Runs through the built-in Hydra-compatible multirun; pick the launcher with
#   hydra/launcher=basic|joblib|gpu_pool   (gpu_pool pins one trial per MI355X).
cd "$(dirname "$0")/.."
python3 train.py -m \
  datamodule=real \
  model=large \
  model.learning_rate=0.001,0.0001,0.00001 \
  trainer.max_epochs=100,200 \
  "$@"
