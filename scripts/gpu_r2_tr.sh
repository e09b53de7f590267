#!/bin/bash
# transformer extras: bench + kernel trace (per-dispatch grid sizes / durations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2t}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 200 python bench.py --model transformer_encoder --steps 100 --warmup 10 > $OUT/bench_tr.jsonl 2> $OUT/bench_tr.err; rc=$?; st "bench rc=$rc"; fatal $rc bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o tr -- python3 bench.py --model transformer_encoder --steps 20 --warmup 5 > $OUT/prof.log 2>&1; rc=$?; st "rocprof rc=$rc"; fatal $rc rocprof
st done
