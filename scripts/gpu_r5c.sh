#!/bin/bash
# r5: restructured pipelined LSTM (backward dx + forward projection in their own workgroups): probe timing, fp64
# parity tests of the LSTM kernels, headline bench and a kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export OUT=${OUT:-r5h}
export SPECS="100 2 3 60 0 1;100 2 1 60 0 1;100 1 3 60 0 0;100 4 3 60 0 3"
export PYTEST=1 PYTEST_K="lstm or test_gpu_kernels" BENCH=1 PROF=1
bash scripts/gpu_probe.sh
