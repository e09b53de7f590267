#!/bin/bash
# Diagnostic binaries (not part of the extension).
#   scripts/build_probes.sh                LSTM stack timing probe and its s_memtime stamp build
#   scripts/build_probes.sh gemm           256 x 256 GEMM probe (timing build + stamp build)
#   scripts/build_probes.sh gemm-variants  the same with schedule variants (A/B builds)
cd "$(dirname "$0")/.."
mkdir -p tools_bin
F="--offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics -I csrc ${EXTRA:-}"
case "$1" in
  gemm)
    hipcc $F csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe &
    hipcc $F -DMTA_GEMM_STAMPS csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe_s &
    ;;
  gemm-variants)
    hipcc $F -DMTA_GEMM_DMA_IN_READS=1 -DMTA_GEMM_BIG_AHEAD=3 csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe_r &
    hipcc $F -DMTA_GEMM_DMA_IN_READS=1 -DMTA_GEMM_BIG_AHEAD=3 -DMTA_GEMM_STAMPS csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe_rs &
    hipcc $F -DMTA_GEMM_NO_PRIO csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe_np &
    hipcc $F -DMTA_GEMM_STATIC_PRIO csrc/tools/gemm_probe.hip -o tools_bin/gemm_probe_sp &
    ;;
  *)
    hipcc $F csrc/tools/lstm_stack_probe.hip -o tools_bin/stack_s0 &
    hipcc $F -DMTA_STACK_STAMPS=1 csrc/tools/lstm_stack_probe.hip -o tools_bin/stack_s1 &
    ;;
esac
wait
