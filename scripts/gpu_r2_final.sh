#!/bin/bash
# round-end rehearsal: what the driver runs (pytest -m gpu, smoke, default bench) + the all-model sweep + headline trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2f}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; st "smoke rc=$rc"; fatal $rc smoke
timeout -k 10 200 python bench.py > $OUT/bench_default.jsonl 2> $OUT/bench_default.err; rc=$?; st "bench default rc=$rc"; fatal $rc bench
R2_OUT=${R2_OUT:-r2f} bash scripts/gpu_r2_sweep.sh; rc=$?; st "sweep rc=$rc"; fatal $rc sweep
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o small -- python3 bench.py --steps 400 --warmup 20 > $OUT/prof.log 2>&1; rc=$?; st "rocprof rc=$rc"; fatal $rc rocprof
st done
