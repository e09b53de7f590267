#!/bin/bash
# 256 x 256 GEMM epilogue probe: the epilogue run twice per tile (cold vs warm instruction cache)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/epi
mkdir -p $O
for b in ${PROBES:-gemm_probe gemm_probe_tw}; do
  for sh in "6400 2048 2048 0 1" "6400 2048 2048 1" "2048 2048 6400 2" "4096 4096 4096 0"; do
    echo "## $b $sh" >> $O/probe2.txt
    MTA_GEMM_SK=0 timeout -k 5 30 ./tools_bin/$b $sh >> $O/probe2.txt 2>&1 || { echo "FATAL $b $sh" >> $O/probe2.txt; exit 1; }
  done
done
