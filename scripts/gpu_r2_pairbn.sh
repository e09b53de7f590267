#!/bin/bash
# 128x64 vs 128x128 tiles for the big paired weight-/input-gradient launch (mlp_large), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-pairbn}
mkdir -p $OUT
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
for v in 0 1 0 1; do
MTA_GEMM_PAIR_BN64=$v timeout -k 10 240 python bench.py --model mlp_large --batch 64 --steps 50 --warmup 5 >> $OUT/mlp_$v.jsonl 2>> $OUT/mlp.err; rc=$?; st "mlp pair_bn64=$v rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
MTA_GEMM_PAIR_BN64=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_extras.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; st "pytest rc=$rc"
exit $rc
