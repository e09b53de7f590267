#!/bin/bash
# round-end evidence, part B: every model's 1-GPU bench, extras kernel traces, trial packing k=2..8
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final_b STEPS=100 PROFILE=1 bash scripts/gpu_bench_all.sh || exit $?
bash scripts/gpu_pack_sweep.sh || exit $?
