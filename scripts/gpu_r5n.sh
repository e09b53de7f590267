#!/bin/bash
# grouped weight-gradient tile / split sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
timeout -k 10 600 python scripts/wgrad_group_bench.py --sweep > $O/sweep.jsonl 2> $O/sweep.err || exit $?
echo done >> $O/status.log
