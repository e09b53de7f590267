#!/bin/bash
# r5w: LSTM fused weight-gradient chunks split over rows at large batch.  The A/B used a temporary
# LSTM_WG_ROWS_PROBE override (removed; the launcher now uses WG_FUSED_MAX_ROWS = 4096).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5w2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm_pipeline.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
for b in 64; do
  for r in 0 3000 4096 0 4096; do
    echo -n "B=$b rows=$r :: " >> $O/ab.log
    LSTM_WG_ROWS_PROBE=$r timeout -k 10 200 python bench.py --model small --loss mse --batch $b --steps 60 --warmup 10 2>/dev/null | python -c "import sys,json; print(json.loads(sys.stdin.readline())['p50_step_ms'])" >> $O/ab.log || exit 1
  done
done
for m in "--model small --loss combined --batch 64" "--model small --loss mse --batch 1"; do
  echo -n "$m default :: " >> $O/ab.log
  timeout -k 10 200 python bench.py $m --steps 100 --warmup 10 2>/dev/null | python -c "import sys,json; print(json.loads(sys.stdin.readline())['p50_step_ms'])" >> $O/ab.log || exit 1
done
echo done >> $O/status.log
