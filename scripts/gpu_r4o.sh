#!/bin/bash
# extras fused training step (one-launch decoder): parity tests, A/B benches (MTA_FUSED_STEP=0 = autograd decoder)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extras.py tests/test_gpu_engine.py -k "fused or extras_fused or engine" > $O/pytest.log 2>&1 || exit $?
for f in 1 0 1 0; do
  MTA_FUSED_STEP=$f timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_tr.jsonl 2>> $O/bench.err || exit $?
  MTA_FUSED_STEP=$f timeout -k 10 300 python bench.py --model mlp_small --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_ms.jsonl 2>> $O/bench.err || exit $?
  MTA_FUSED_STEP=$f timeout -k 10 300 python bench.py --model mlp_small --trainer fast --steps 200 --warmup 20 >> $O/bench_msf.jsonl 2>> $O/bench.err || exit $?
done
