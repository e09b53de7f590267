#!/bin/bash
# producers after the float4-aligned flat layout: bookkeeping trace, the whole GPU suite, mlp_large A/B + trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 200 python -u scripts/wgrad_split_sweep.py > $O/wgrad_split.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/debug_producers.py > $O/debug_producers.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for f in 1 0 1 0; do
  MTA_OPTIM_PRODUCERS=$f timeout -k 10 300 python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 100 --warmup 10 >> $O/bench_mlp.jsonl 2>> $O/bench.err || exit $?
done
MTA_OPTIM_PRODUCERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 92 --warmup 10 > $O/prof_mlp.log 2>&1 || exit $?
