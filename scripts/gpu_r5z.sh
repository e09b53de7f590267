#!/bin/bash
# r5z: transformer weight gradients grouped at any K: tests, B=8 / B=1 bench, B=8 trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_extras.py tests/test_gpu_graphs.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
timeout -k 10 300 python bench.py --model transformer_encoder --loss combined --batch 8 --trainer gpu_fast --steps 100 --warmup 10 > $O/tr_b8.json 2> $O/tr_b8.err || { echo "bench rc=$?" >> $O/status.log; exit 1; }
timeout -k 10 300 python bench.py --model transformer_encoder --loss mse --batch 1 --trainer gpu_fast --steps 200 --warmup 20 > $O/tr_b1.json 2> $O/tr_b1.err || { echo "bench rc=$?" >> $O/status.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tr8 -o tr8 -- python bench.py --model transformer_encoder --loss combined --batch 8 --trainer gpu_fast --steps 30 --warmup 5 > $O/prof_tr8.log 2>&1 || { echo "prof rc=$?" >> $O/status.log; exit 1; }
echo done >> $O/status.log
