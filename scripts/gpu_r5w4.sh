#!/bin/bash
# r5w4: LSTM B=8/16/64 A/B of the fused weight-gradient row split (used a temporary LSTM_WG_ROWS_PROBE
# override, since removed: the launcher now always splits chunks above WG_FUSED_SPLIT_ROWS in two)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5w5
mkdir -p $O
for b in 16 64 8; do
  for r in 4096 -512 4096 -512; do
    echo -n "B=$b rows=$r :: " >> $O/ab.log
    LSTM_WG_ROWS_PROBE=$r timeout -k 10 200 python bench.py --model small --loss mse --batch $b --steps 100 --warmup 10 2>/dev/null | python -c "import sys,json; print(json.loads(sys.stdin.readline())['p50_step_ms'])" >> $O/ab.log || exit 1
  done
done
echo done >> $O/status.log
