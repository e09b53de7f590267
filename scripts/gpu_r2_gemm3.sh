#!/bin/bash
# GEMM tests + BK128 A/B + extras benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-gemm3}
mkdir -p $OUT
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_extras.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; st "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
MTA_GEMM_BK128=1 timeout -k 10 240 python -u scripts/gemm_bench.py > $OUT/gemm_bk128.log 2>&1; rc=$?; st "gemm bk128 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python -u scripts/gemm_bench.py --json $OUT/gemm.jsonl > $OUT/gemm.log 2>&1; rc=$?; st "gemm rc=$rc"; [ $rc -ne 0 ] && exit $rc
MTA_GEMM_BK128=1 timeout -k 10 240 python bench.py --model mlp_large --batch 64 --steps 30 --warmup 5 > $OUT/mlp_bk128.jsonl 2> $OUT/mlp.err; rc=$?; st "mlp bk128 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --model mlp_large --batch 64 --steps 30 --warmup 5 > $OUT/mlp.jsonl 2> $OUT/mlp.err; rc=$?; st "mlp rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --model transformer_encoder --batch 1 --steps 100 --warmup 10 > $OUT/tr.jsonl 2> $OUT/tr.err; rc=$?; st "tr rc=$rc"
exit $rc
