#!/bin/bash
# fused attention split into query halves (MTA_TR_ATTN_SPLIT): parity tests, transformer A/B, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
MTA_TR_ATTN_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extras.py -k "transformer or attention" > $O/pytest.log 2>&1 || exit $?
for f in 1 0 1 0; do
  MTA_TR_ATTN_SPLIT=$f timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_tr.jsonl 2>> $O/bench.err || exit $?
done
MTA_TR_ATTN_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tr -o tr -- python bench.py --model transformer_encoder --trainer gpu_fast --steps 50 --warmup 10 > $O/prof_tr.log 2>&1 || exit $?
