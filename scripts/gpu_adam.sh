#!/bin/bash
# Fused Adam streaming-path check: optimizer GPU tests, mlp_large B=64 bench and its kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k adam \
  > $OUT/pytest_adam.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --model mlp_large --loss mse --batch 64 --trainer gpu_fast --steps 100 --warmup 10 \
  > $OUT/bench_mlp_large.json 2> $OUT/bench_mlp_large.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mlp -o mlp -- \
  python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 50 --warmup 10 > $OUT/prof_mlp.log 2>&1 || exit $?
