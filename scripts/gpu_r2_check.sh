#!/bin/bash
# GPU tests + headline bench + kernel trace of the headline step (round-2 iteration check).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2c}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
st pytest
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
st bench
timeout -k 10 120 python bench.py --steps 500 --warmup 50 > $OUT/bench.jsonl 2> $OUT/bench.err; rc=$?; st "bench rc=$rc"; fatal $rc bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o small -- python bench.py --steps 200 --warmup 20 > $OUT/prof.log 2>&1; rc=$?; st "rocprof rc=$rc"; fatal $rc rocprof
st done
