#!/bin/bash
# fused FFN half: timing + phase stamps.  Build first:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc -DMTA_STAMPS=1 \
#         csrc/tools/ffn_probe.hip -o tools_bin/ffn_probe_1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ffnp
mkdir -p $O
timeout -k 10 60 ./tools_bin/ffn_probe_1 > $O/ffn_probe.log 2>&1 || exit $?
