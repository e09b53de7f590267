#!/bin/bash
# r5z: double-buffered Adam streaming loop: optimizer / kernel tests, mlp_large bench + trace, headline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5z
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_extras.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
timeout -k 10 300 python bench.py --model mlp_large --loss mse --batch 64 --trainer gpu_fast --steps 100 --warmup 10 > $O/mlp_large.json 2> $O/mlp_large.err || { echo "bench rc=$?" >> $O/status.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 50 --warmup 10 > $O/prof_mlp.log 2>&1 || { echo "prof rc=$?" >> $O/status.log; exit 1; }
echo done >> $O/status.log
