#!/bin/bash
# r5x: in-kernel split-K reduction (weight-gradient shape): old build / separate reduce (3) / in-kernel (-1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5x
mkdir -p $O
for i in 1 2; do
  for v in "gemm_probe_old 2048 2048 6400 2 0 4" "gemm_probe 2048 2048 6400 2 0 4 3" "gemm_probe 2048 2048 6400 2 0 4 -1" "gemm_probe 1032 776 4032 2 0 11 -1"; do
    echo -n "$v :: " >> $O/probe_red.log
    set -- $v
    b=$1; shift
    timeout -k 5 60 probe_bin/$b "$@" >> $O/probe_red.log 2>&1 || exit 1
  done
done
echo done >> $O/probe_red.log
