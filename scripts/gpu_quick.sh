#!/bin/bash
# Quick GPU iteration: GPU tests (-x), microbench, bench; optional rocprof (PROFILE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
echo "start $(date)" > $OUT/status.log
fatal() { case "$1" in 0|1) return 0;; *) echo "FATAL $2 rc=$1" >> $OUT/status.log; exit "$1";; esac; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $OUT/status.log; fatal $rc pytest
if [ -n "$MICRO" ]; then timeout -k 10 600 python scripts/microbench.py > $OUT/micro.log 2>&1; rc=$?; echo "micro rc=$rc" >> $OUT/status.log; fatal $rc micro; fi
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-200} --warmup 20 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?; echo "bench rc=$rc" >> $OUT/status.log; fatal $rc bench
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python bench.py --steps 100 --warmup 20 ${BENCH_ARGS:-} > $OUT/prof_bench.log 2>&1; rc=$?; echo "rocprof rc=$rc" >> $OUT/status.log; fatal $rc rocprof
fi
echo "done $(date)" >> $OUT/status.log
