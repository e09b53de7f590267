#!/bin/bash
# register-resident fused Adam: float4 per thread (MTA_ADAM_REG_PER) A/B on the headline; optimizer tests at 2 and 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
for per in 2 4; do
  MTA_ADAM_REG_PER=$per timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k adam > $O/pytest_$per.log 2>&1 || exit $?
done
for per in 1 2 4 1 2 4; do
  MTA_ADAM_REG_PER=$per timeout -k 10 300 python bench.py > $O/h_$per.json 2>> $O/bench.err || exit $?
  echo "$per $(cat $O/h_$per.json)" >> $O/sweep.txt
done
