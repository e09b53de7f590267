#!/bin/bash
# GEMM probe session (build the binaries with scripts/build_probes.sh gemm first): timing + stamp split of the
# 256 x 256 kernel on the mlp_large shapes and 4096^3.  OUT=<subdir of gpurun_out>  PROBES="gemm_probe ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-gp}
mkdir -p $OUT
for b in ${PROBES:-gemm_probe gemm_probe_s}; do
  for sh in "4096 4096 4096 0" "6400 2048 2048 0 1" "6400 2048 2048 1" "2048 2048 6400 2"; do
    timeout -k 5 30 ./tools_bin/$b $sh >> $OUT/probe.txt 2>&1 || { echo "FATAL $b $sh" >> $OUT/probe.txt; exit 1; }
  done
done
