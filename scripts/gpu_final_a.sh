#!/bin/bash
# round-end evidence, part A: the whole GPU test suite, then the headline bench (3 runs) and its kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py >> $O/bench_headline.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_small -o small -- python bench.py --steps 100 --warmup 20 > $O/prof_small.log 2>&1 || exit $?
