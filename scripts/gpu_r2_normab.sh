#!/bin/bash
# transformer step with the narrow norm backward's grid cap at 512 / 1024 blocks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-normab}
mkdir -p $OUT
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
for cap in 1024 1568 1024 1568; do
MTA_NORM_BWD_BLOCKS=$cap timeout -k 10 240 python bench.py --model transformer_encoder --batch 1 --steps 200 --warmup 10 >> $OUT/tr_$cap.jsonl 2> $OUT/tr.err; rc=$?; st "tr cap=$cap rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
MTA_NORM_BWD_BLOCKS=1568 timeout -k 10 240 python -u -m pytest tests/test_gpu_extras.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; st "pytest rc=$rc"
exit $rc
