#!/bin/bash
# Thesis grid on synthetic data: 3 models x 3 losses x 2 trainers = 18 jobs.
# On an 8-GPU node run the trials concurrently, one per GPU:
#   bash sweeps/experiment_synthetic.sh hydra/launcher=gpu_pool
cd "$(dirname "$0")/.."
python3 train.py -m \
  datamodule=synthetic \
  model=small,medium,large \
  loss=mse,nll,combined \
  trainer=fast,slow \
  "$@"
