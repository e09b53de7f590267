#!/bin/bash
# quick iteration: selected GPU tests (PYTEST_K / PYTEST_FILES) + headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2q}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 600 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python bench.py --steps 500 --warmup 50 > $OUT/bench.jsonl 2> $OUT/bench.err; rc=$?; st "bench rc=$rc"; fatal $rc bench
st done
