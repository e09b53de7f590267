#!/bin/bash
# Round-2 first GPU session: all GPU tests (incl. the train.py -> test.py product run), headline bench,
# same-node PyTorch (MIOpen) reference-path benches, headline rocprof kernel trace.
# Any signal / timeout exit ends the script (no further GPU work after a fault).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2a
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
st pytest
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
st bench
timeout -k 10 120 python bench.py --steps 500 --warmup 50 > $OUT/bench_small.jsonl 2> $OUT/bench_small.err; rc=$?; st "bench rc=$rc"; fatal $rc bench
for spec in "small 1" "medium 1" "large 1" "small 8" "small 64"; do
  set -- $spec
  for g in "" "--no-graphs"; do
    timeout -k 10 300 python bench.py --backend torch --model $1 --batch $2 --steps 100 --warmup 10 $g >> $OUT/bench_torch.jsonl 2>> $OUT/bench_torch.err; rc=$?; st "torch $spec $g rc=$rc"; fatal $rc torch
  done
  timeout -k 10 120 python bench.py --model $1 --batch $2 --steps 300 --warmup 30 >> $OUT/bench_hip.jsonl 2>> $OUT/bench_hip.err; rc=$?; st "hip $spec rc=$rc"; fatal $rc hip
done
st rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o small -- python bench.py --steps 200 --warmup 20 > $OUT/prof.log 2>&1; rc=$?; st "rocprof rc=$rc"; fatal $rc rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_torch -o torch -- python bench.py --backend torch --steps 100 --warmup 10 > $OUT/prof_torch.log 2>&1; rc=$?; st "rocprof torch rc=$rc"; fatal $rc rocprof_torch
st done
