#!/bin/bash
# pipelined 64x64x128 NN tiles (MTA_GEMM_PIPE64): correctness with it on, wgrad split sweep and transformer A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
MTA_GEMM_PIPE64=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extras.py -k "transformer or ffn or gemm or paired" > $O/pytest.log 2>&1 || exit $?
for f in 1 0; do
  MTA_GEMM_PIPE64=$f timeout -k 10 200 python -u scripts/wgrad_split_sweep.py > $O/sweep_$f.log 2>&1 || exit $?
done
for f in 1 0 1 0; do
  MTA_GEMM_PIPE64=$f timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_tr.jsonl 2>> $O/bench.err || exit $?
done
