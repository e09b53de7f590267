#!/bin/bash
# bf16 wide rows for the MLP (GEMM epilogue -> norm): mlp_large bench + trace; Adam two-launch A/B; extras tests;
# transformer with the operand casts riding on the packing launch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 300 python bench.py --model mlp_large --loss mse --batch 64 --trainer gpu_fast --steps 100 --warmup 10 \
  > $O/mlp_large.json 2> $O/mlp_large.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- \
  python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 50 --warmup 10 > $O/prof_mlp.log 2>&1 || exit $?
for m in "--model small" "--model transformer_encoder --trainer gpu_fast"; do
  for two in 0 1; do
    MTA_OPTIM_TWO_LAUNCH=$two timeout -k 10 200 python bench.py $m --steps 200 --warmup 20 >> $O/adam_ab.jsonl \
      2>> $O/adam_ab.err || exit $?
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_extras.py -m gpu -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/status.log
timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 \
  > $O/transformer.json 2> $O/transformer.err || exit $?
echo done >> $O/status.log
