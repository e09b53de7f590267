#!/bin/bash
# Accuracy against the thesis' published numbers: the thesis set-up (`tex/diplomski_rad.tex:1099-1126`:
# synthetic, 10,000 windows of 100 stocks, H=32, plateau x0.5 / 2, early stopping 10, ΔL reporting) for the three
# losses at the default 32-true matmul precision ("high") and at "highest", three trainers at a time on one MI355X;
# then test.py on each run's best checkpoint for the alpha / beta / reconstruction correlations.
#   bash scripts/gpu_thesis.sh [max_epochs]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/thesis
mkdir -p $O
EP=${1:-120}
COMMON="datamodule.n_samples=900000 seed=0 model.hidden_size=32 model.num_layers=2 model.learning_rate=0.001"
export MTA_LSTM_SPIN_LIMIT=$((1 << 25)) MTA_ADAM_SPIN_LIMIT=$((1 << 26)) GPU_MAX_HW_QUEUES=1
for P in high highest; do
  pids=()
  for L in mse nll combined; do
    timeout -k 10 900 python -u train.py $COMMON trainer=thesis trainer.max_epochs=$EP loss=$L \
      +trainer.matmul_precision=$P report_delta=true test_ckpt=best trainer.devices=1 \
      logger.version=thesis_${L}_${P} > $O/train_${L}_${P}.log 2>&1 &
    pids+=($!)
  done
  for p in "${pids[@]}"; do wait $p || { echo "train failed rc=$?" >> $O/status.log; exit 1; }; done
  echo "[$(date +%T)] $P trained" >> $O/status.log
done
for P in high highest; do
  for L in mse nll combined; do
    ck=$(grep -o "Best model path: .*" $O/train_${L}_${P}.log | head -1 | cut -d' ' -f4-)
    timeout -k 10 300 python -u test.py $COMMON loss=$L checkpoint=$ck +device=cuda > $O/test_${L}_${P}.log 2>&1 \
      || { echo "test failed $L $P" >> $O/status.log; exit 1; }
  done
done
python scripts/thesis_summary.py $O > $O/thesis_accuracy.jsonl
echo "[$(date +%T)] done" >> $O/status.log
