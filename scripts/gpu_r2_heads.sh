#!/bin/bash
# kernel tests (wide heads path) + mlp_large trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-heads}
mkdir -p $OUT
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_extras.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; st "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 python bench.py --model mlp_large --batch 64 --steps 50 --warmup 5 > $OUT/mlp.jsonl 2> $OUT/mlp.err; rc=$?; st "mlp rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o mlp -- python3 bench.py --model mlp_large --batch 64 --steps 20 --warmup 5 > $OUT/prof.log 2>&1; rc=$?; st "rocprof rc=$rc"
exit $rc
