#!/bin/bash
# fused FFN half: timing + phase stamps, and the two load-removal experiments (weights, x1 rows).  Build first:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc -DMTA_FFN_STAMPS=1 [-DMTA_FFN_EXP=1|2] \
#         csrc/tools/ffn_probe.hip -o tools_bin/ffn_probe_1 (ffn_probe_e1 / ffn_probe_e2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ffnp
mkdir -p $O
{ timeout -k 10 60 ./tools_bin/ffn_probe_1 && echo "## EXP 1: no weight-fragment loads" && timeout -k 10 60 ./tools_bin/ffn_probe_e1 \
  && echo "## EXP 2: no x1 row loads" && timeout -k 10 60 ./tools_bin/ffn_probe_e2; } > $O/ffn_probe_exp.log 2>&1 || exit $?
