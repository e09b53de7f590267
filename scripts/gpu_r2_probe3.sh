#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2j}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
for spec in "100 2 1 60 0 1" "100 2 1 60 0 0" "100 4 1 60 0 3" "6400 2 1 60 0 1"; do
  timeout -k 10 90 ./tools_bin/stack_s1 $spec >> $OUT/probe.txt 2>&1; rc=$?; st "probe $spec rc=$rc"; fatal $rc probe
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "lstm or engine" > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
for b in 1 8 64; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --batch $b >> $OUT/bench.jsonl 2>> $OUT/bench.err; rc=$?; st "bench B=$b rc=$rc"; fatal $rc bench
done
st done
