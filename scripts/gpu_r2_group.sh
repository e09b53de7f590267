#!/bin/bash
# grouped step graphs: engine tests, bench S=1 vs S=8 (B=1, 8), kernel trace of the grouped headline step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2g}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-engine or e2e}" > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
for b in 1 8; do
  for S in 1 8 16; do
    timeout -k 10 180 python bench.py --steps 400 --warmup 20 --batch $b --steps-per-graph $S >> $OUT/bench.jsonl 2>> $OUT/bench.err; rc=$?; st "bench B=$b S=$S rc=$rc"; fatal $rc bench
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 400 --warmup 20 --batch 1 > $OUT/prof_bench.log 2>&1; rc=$?; st "rocprof rc=$rc"; fatal $rc rocprof
st done
