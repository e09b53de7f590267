#!/bin/bash
# streaming fused Adam (unrolled loads): optimizer tests, mlp_large bench x2 + kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "adam" > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 100 --warmup 10 >> $O/bench_mlp.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 50 --warmup 10 > $O/prof_mlp.log 2>&1 || exit $?
