#!/bin/bash
# cheaper norm dropout hash; transformer embedding fused into the first attention half + casts riding on frag_pack
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_extras.py tests/test_gpu_graphs.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
timeout -k 10 300 python bench.py --model mlp_large --loss mse --batch 64 --trainer gpu_fast --steps 100 --warmup 10 \
  > $O/mlp_large.json 2> $O/mlp_large.err || exit $?
timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 \
  > $O/transformer.json 2> $O/transformer.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- \
  python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 50 --warmup 10 > $O/prof_mlp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tr -o tr -- \
  python bench.py --model transformer_encoder --trainer gpu_fast --steps 50 --warmup 10 > $O/prof_tr.log 2>&1 || exit $?
echo done >> $O/status.log
