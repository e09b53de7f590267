#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${R2_OUT:-r2k}
mkdir -p $OUT
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
for d in 0 4 8 12; do
  for spec in "100 2 1 60 0" "100 4 1 60 0" "800 2 1 60 0"; do
    timeout -k 10 90 ./tools_bin/stack_d$d $spec >> $OUT/probe.txt 2>&1; rc=$?; echo "d=$d $spec rc=$rc" >> $OUT/status.log; fatal $rc probe
  done
done
