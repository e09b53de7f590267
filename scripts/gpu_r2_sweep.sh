#!/bin/bash
# end-of-session sweep: headline + batch sweep + medium/large + extras, one JSON line each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2s}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
run() { timeout -k 10 240 python bench.py "$@" >> $OUT/sweep.jsonl 2>> $OUT/sweep.err; rc=$?; st "bench $* rc=$rc"; fatal $rc bench; }
run --steps 1000 --warmup 50
run --steps 400 --warmup 20 --batch 8
run --steps 100 --warmup 10 --batch 64
run --steps 400 --warmup 20 --model medium
run --steps 400 --warmup 20 --model large
run --steps 400 --warmup 20 --loss nll
run --steps 400 --warmup 20 --loss combined
run --steps 100 --warmup 10 --model transformer_encoder
run --steps 100 --warmup 10 --model transformer_encoder --batch 8
run --steps 200 --warmup 10 --model mlp_small
run --steps 50 --warmup 5 --model mlp_large --batch 64
st done
