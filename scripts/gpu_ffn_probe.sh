#!/bin/bash
# fused FFN half: timing + phase stamps, and the two load-removal experiments (weights, x1 rows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ffnp
mkdir -p $O
{ timeout -k 10 60 ./tools_bin/ffn_probe_1 && echo "## EXP 1: no weight-fragment loads" && timeout -k 10 60 ./tools_bin/ffn_probe_e1 \
  && echo "## EXP 2: no x1 row loads" && timeout -k 10 60 ./tools_bin/ffn_probe_e2; } > $O/ffn_probe_exp.log 2>&1 || exit $?
