#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2y}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_extras.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
for spec in "transformer_encoder 1" "transformer_encoder 8" "mlp_large 64"; do
  set -- $spec
  timeout -k 10 240 python bench.py --model $1 --batch $2 --steps 100 --warmup 10 >> $OUT/bench.jsonl 2>> $OUT/bench.err; rc=$?; st "bench $spec rc=$rc"; fatal $rc bench
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_tr1 -o tr1 -- python bench.py --model transformer_encoder --batch 1 --steps 50 --warmup 10 > $OUT/prof_tr1.log 2>&1; rc=$?; st "prof tr1 rc=$rc"; fatal $rc prof
R2_OUT=${R2_OUT:-r2y}/pmc bash scripts/gpu_r2_pmc.sh
st done
