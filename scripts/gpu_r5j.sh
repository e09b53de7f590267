#!/bin/bash
# 32-true transformer on HIP (gemm_f32x epilogues + attention_f32): extras GPU tests, then more thesis-accuracy runs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_extras.py -m gpu -x -v --timeout 200 --timeout-method thread \
  -k "32true or honour" > $O/pytest_f32.log 2>&1 || { echo "pytest rc=$?" >> $O/status.log; exit 1; }
echo "pytest ok" >> $O/status.log
bash scripts/gpu_thesis.sh 100 highest 0 && bash scripts/gpu_thesis.sh 100 high 1
