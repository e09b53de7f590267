#!/bin/bash
# North-star extras (not in the reference): MLP / transformer encoders, bf16-mixed, all losses.
cd "$(dirname "$0")/.."
python3 train.py -m \
  datamodule=synthetic \
  model=mlp_small,mlp_large,transformer_encoder \
  loss=mse,nll,combined \
  trainer=gpu_fast \
  "$@"
