#!/bin/bash
# Accuracy against the thesis' published numbers: the thesis set-up (`tex/diplomski_rad.tex:1099-1126`:
# synthetic, 10,000 windows of 100 stocks, H=32, plateau x0.5 / 2, early stopping 10, ΔL reporting) for the three
# losses at the default 32-true matmul precision ("high") and/or "highest", one trainer at a time (trainers
# time-slicing one GPU stall the pipelined LSTM's cross-workgroup hand-offs past their spin limit); then test.py on
# each run's best checkpoint for the alpha / beta / reconstruction correlations.
#   bash scripts/gpu_thesis.sh [max_epochs] [precisions, default "high highest"] [seeds, default "0"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/thesis
mkdir -p $O
EP=${1:-120}
PRECS=${2:-high highest}
SEEDS=${3:-0}
COMMON="datamodule.n_samples=900000 model.hidden_size=32 model.num_layers=2 model.learning_rate=0.001"
for S in $SEEDS; do
for P in $PRECS; do
  for L in mse nll combined; do
    R=${L}_${P}_s${S}
    timeout -k 10 420 python -u train.py $COMMON seed=$S trainer=thesis trainer.max_epochs=$EP loss=$L \
      +trainer.matmul_precision=$P report_delta=true test_ckpt=best trainer.devices=1 \
      logger.version=thesis_$R > $O/train_$R.log 2>&1 \
      || { echo "train failed $R rc=$?" >> $O/status.log; exit 1; }
    ck=$(grep -o "Best model path: .*" $O/train_$R.log | head -1 | cut -d' ' -f4-)
    timeout -k 10 300 python -u test.py $COMMON seed=$S loss=$L checkpoint=$ck +device=cuda > $O/test_$R.log 2>&1 \
      || { echo "test failed $R" >> $O/status.log; exit 1; }
    echo "[$(date +%T)] $R done" >> $O/status.log
  done
done
done
python scripts/thesis_summary.py $O > $O/thesis_accuracy.jsonl
echo "[$(date +%T)] done" >> $O/status.log
