#!/bin/bash
# Stack-probe matrix (mode / precision) + LSTM GPU tests + headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2h}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
for spec in "100 2 1 60 0" "100 2 1 60 1" "100 2 1 60 2" "100 2 2 60 0" "100 2 0 60 0"; do
  for b in stack_s0 stack_s1; do
    timeout -k 10 60 ./tools_bin/$b $spec >> $OUT/probe.txt 2>&1; rc=$?; st "$b $spec rc=$rc"; fatal $rc $b
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "lstm or engine" > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
timeout -k 10 120 python bench.py --steps 500 --warmup 50 > $OUT/bench.jsonl 2> $OUT/bench.err; rc=$?; st "bench rc=$rc"; fatal $rc bench
st done
