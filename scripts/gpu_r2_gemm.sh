#!/bin/bash
# GEMM micro-benchmark + mlp_large / transformer kernel traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-gemm}
mkdir -p $OUT
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 240 python -u scripts/gemm_bench.py --json $OUT/gemm.jsonl > $OUT/gemm.log 2>&1; rc=$?; st "gemm rc=$rc"; [ $rc -ne 0 ] && exit $rc
if [ -n "$GEMM_ONLY" ]; then exit 0; fi
timeout -k 10 240 python bench.py --model mlp_large --batch 64 --steps 30 --warmup 5 > $OUT/mlp.jsonl 2> $OUT/mlp.err; rc=$?; st "mlp rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --model transformer_encoder --batch 1 --steps 100 --warmup 10 > $OUT/tr.jsonl 2> $OUT/tr.err; rc=$?; st "tr rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o mlp -- python3 bench.py --model mlp_large --batch 64 --steps 20 --warmup 5 > $OUT/prof.log 2>&1; rc=$?; st "rocprof rc=$rc"
exit $rc
