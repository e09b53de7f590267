#!/bin/bash
# Diagnostic binaries (not part of the extension): LSTM stack timing probe and its s_memtime stamp build.
cd "$(dirname "$0")/.."
mkdir -p tools_bin
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc ${EXTRA:-} csrc/tools/lstm_stack_probe.hip -o tools_bin/stack_s0 &
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc ${EXTRA:-} -DMTA_STACK_STAMPS=1 csrc/tools/lstm_stack_probe.hip -o tools_bin/stack_s1 &
wait
