#!/bin/bash
# r5z: grid losses from N = 512: kernel tests, LSTM / transformer B=8 bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5z2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
for m in "--model small --loss mse --batch 8" "--model small --loss combined --batch 8" "--model transformer_encoder --loss combined --batch 8 --trainer gpu_fast"; do
  echo -n "$m :: " >> $O/b8.log
  timeout -k 10 200 python bench.py $m --steps 100 --warmup 10 2>/dev/null | python -c "import sys,json; print(json.loads(sys.stdin.readline())['p50_step_ms'])" >> $O/b8.log || exit 1
done
echo done >> $O/status.log
