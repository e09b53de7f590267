#!/bin/bash
# fused transformer FFN: extras tests, transformer bench fused / unfused, mlp_large bench, kernel trace of the transformer
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ffn
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_extras.py > $O/pytest.log 2>&1 || exit $?
for f in 1 0; do
  MTA_TR_FFN=$f MTA_TR_ATTN=$f timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 300 python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 100 --warmup 10 >> $O/bench.jsonl 2>> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o tr -- python bench.py --model transformer_encoder --trainer gpu_fast --steps 92 --warmup 10 > $O/prof.log 2>&1 || exit $?
