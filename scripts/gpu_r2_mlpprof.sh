#!/bin/bash
# mlp_large kernel traces, pipelined GEMM main loop off / on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-mlpprof}
mkdir -p $OUT
export TMPDIR=/tmp
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
MTA_GEMM_PIPE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof0 -o mlp -- python3 bench.py --model mlp_large --batch 64 --steps 20 --warmup 5 > $OUT/prof0.log 2>&1; rc=$?; st "rocprof0 rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof1 -o mlp -- python3 bench.py --model mlp_large --batch 64 --steps 20 --warmup 5 > $OUT/prof1.log 2>&1; rc=$?; st "rocprof1 rc=$rc"
exit $rc
