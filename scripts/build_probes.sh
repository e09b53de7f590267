#!/bin/bash
# Diagnostic binaries (not part of the extension).
#   scripts/build_probes.sh                LSTM stack timing probe and its s_memtime stamp build
#   scripts/build_probes.sh gemm           256 x 256 GEMM probe (timing build + stamp build)
cd "$(dirname "$0")/.."
mkdir -p tools_bin
F="--offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc ${EXTRA:-}"
case "$1" in
  gemm)
    hipcc $F csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe &
    hipcc $F -DMTA_STAMPS=1 csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe_s &
    ;;
  *)
    hipcc $F csrc/tools/lstm_stack_probe.hip -o tools_bin/stack_s0 &
    hipcc $F -DMTA_STAMPS=1 csrc/tools/lstm_stack_probe.hip -o tools_bin/stack_s1 &
    hipcc $F -DMTA_STAMPS=2 csrc/tools/lstm_stack_probe.hip -o tools_bin/stack_tl &
    ;;
esac
wait
