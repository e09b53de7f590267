#!/bin/bash
# kernel trace of the headline bench (B=1) for per-step kernel durations and inter-kernel gaps
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2p}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 python bench.py --steps 200 --warmup 20 --batch ${BENCH_B:-1} > $OUT/bench_plain.jsonl 2> $OUT/bench_plain.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 200 --warmup 20 --batch ${BENCH_B:-1} > $OUT/bench.log 2>&1; rc=$?
echo "rocprof rc=$rc" | tee -a $OUT/status.log
exit $rc
