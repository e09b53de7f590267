#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2z}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_extras.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
for spec in "transformer_encoder 1 device" "small 64 device" "small 64 stream"; do
  set -- $spec
  timeout -k 10 240 python bench.py --model $1 --batch $2 --residency $3 --steps 100 --warmup 10 >> $OUT/bench.jsonl 2>> $OUT/bench.err; rc=$?; st "bench $spec rc=$rc"; fatal $rc bench
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_tr1 -o tr1 -- python bench.py --model transformer_encoder --batch 1 --steps 30 --warmup 10 > $OUT/prof_tr1.log 2>&1; rc=$?; st "prof tr1 rc=$rc"; fatal $rc prof
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT/prof_stream -o stream -- python bench.py --batch 64 --residency stream --steps 30 --warmup 5 > $OUT/prof_stream.log 2>&1; rc=$?; st "prof stream rc=$rc"; fatal $rc prof
st done
