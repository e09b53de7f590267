#!/bin/bash
# r5w6: LSTM tests + small B=1/8/64 bench after the two-way fused weight-gradient row split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5w6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm_pipeline.py tests/test_gpu_engine.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
for b in 1 8 16 64; do
  echo -n "B=$b :: " >> $O/ab.log
  timeout -k 10 200 python bench.py --model small --loss mse --batch $b --steps 100 --warmup 10 2>/dev/null | python -c "import sys,json; print(json.loads(sys.stdin.readline())['p50_step_ms'])" >> $O/ab.log || exit 1
done
echo done >> $O/status.log
