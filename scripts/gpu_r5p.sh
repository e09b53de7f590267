#!/bin/bash
# fused attention-half backward GEMMs (dO, dxn + RMSNorm1): extras tests, transformer bench + trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_extras.py tests/test_gpu_graphs.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 \
  > $O/transformer.json 2> $O/transformer.err || exit $?
timeout -k 10 300 python bench.py --model transformer_encoder --loss combined --batch 8 --trainer gpu_fast --steps 100 \
  --warmup 10 > $O/transformer_b8.json 2> $O/transformer_b8.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tr -o tr -- \
  python bench.py --model transformer_encoder --trainer gpu_fast --steps 50 --warmup 10 > $O/prof_tr.log 2>&1 || exit $?
echo done >> $O/status.log
