#!/bin/bash
# LSTM stack probe session: stamp / timing probes (tools_bin/stack_s0 = timing build, stack_s1 = s_memtime
# stamp build; build both with scripts/build_probes.sh first), then optional GPU tests and headline bench.
# OUT=<subdir of gpurun_out>  SPECS="N L prec T mode [stamp-layer];..."  PYTEST=1 [PYTEST_K=expr]  BENCH=1  PROF=1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-probe}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ne 0 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
IFS=';' read -ra SPEC_LIST <<< "${SPECS:-100 2 1 60 0 1;100 2 1 60 0 0}"
for spec in "${SPEC_LIST[@]}"; do
  for b in ${PROBES:-stack_s0 stack_s1}; do
    timeout -k 10 90 ./tools_bin/$b $spec >> $OUT/probe.txt 2>&1; rc=$?; st "$b $spec rc=$rc"; fatal $rc "$b $spec"
  done
done
if [ -n "$PYTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
fi
if [ -n "$BENCH" ]; then
  for b in ${BENCH_BATCHES:-1}; do
    timeout -k 10 180 python bench.py --steps 200 --warmup 20 --batch $b ${BENCH_ARGS:-} >> $OUT/bench.jsonl 2>> $OUT/bench.err; rc=$?; st "bench B=$b rc=$rc"; fatal $rc bench
  done
fi
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o prof -- python bench.py --steps 100 --warmup 20 ${BENCH_ARGS:-} > $OUT/prof.log 2>&1; rc=$?; st "rocprof rc=$rc"; fatal $rc rocprof
fi
st done
