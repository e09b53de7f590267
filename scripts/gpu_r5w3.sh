#!/bin/bash
# r5w3: whole GPU suite + LSTM small B=64 bench and kernel trace after the fused weight-gradient row split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${R5W_TAG:-r5w3}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
timeout -k 10 200 python bench.py --model small --loss mse --batch 64 --steps 60 --warmup 10 > $O/b64.json 2> $O/b64.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o b64 -- python3 bench.py --model small --loss mse --batch 64 --steps 30 --warmup 5 > $O/prof.log 2>&1 || exit 1
echo done >> $O/status.log
