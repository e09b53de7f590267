#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2w}
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
for a in "100 0" "100 1"; do
  for b in losses_s0 losses_s1; do timeout -k 10 60 ./tools_bin/$b $a >> $OUT/loss_probe.txt 2>&1; rc=$?; st "$b $a rc=$rc"; fatal $rc lp; done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_extras.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
timeout -k 10 240 python bench.py --model transformer_encoder --batch 1 --steps 100 --warmup 10 >> $OUT/bench.jsonl 2>> $OUT/bench.err; rc=$?; st "bench rc=$rc"; fatal $rc bench
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_tr1 -o tr1 -- python bench.py --model transformer_encoder --batch 1 --steps 30 --warmup 10 > $OUT/prof_tr1.log 2>&1; rc=$?; st "prof tr1 rc=$rc"; fatal $rc prof
st done
