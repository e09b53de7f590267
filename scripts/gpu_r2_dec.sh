#!/bin/bash
# training-decoder rewrite check: old (wave-per-sequence) vs new (thread-per-sequence) probe values + timing,
# the decoder / fused-step GPU tests, and the headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2w}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
for b in losses_reg0 losses_reg1; do
  for nll in 0 1; do for NN in 100 37; do
    timeout -k 10 60 ./tools_bin/$b $NN $nll >> $OUT/probe.txt 2>&1; rc=$?; st "$b $NN $nll rc=$rc"; fatal $rc probe; done
  done
done
timeout -k 10 60 ./tools_bin/losses_reg1 1000 1 >> $OUT/probe.txt 2>&1; rc=$?; st "tps1 N=1000 rc=$rc"; fatal $rc probe
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYTEST_K:-loss or decoder or engine or heads}" > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
for b in ${BENCH_B:-1 8}; do
  timeout -k 10 180 python bench.py --steps 200 --warmup 20 --batch $b >> $OUT/bench.jsonl 2>> $OUT/bench.err; rc=$?; st "bench B=$b rc=$rc"; fatal $rc bench
done
st done
