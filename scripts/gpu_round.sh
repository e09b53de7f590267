#!/bin/bash
# One GPU session: build, GPU tests, 2-rank gloo rehearsal, every-model bench (+ rocprof), headline rocprof.
# Stops at the first failing step (no further GPU work after a fault / timeout).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
step() { echo "[gpu_round] $1" >&2; }
step build
python -m masters_thesis_amd.ops.build > gpurun_out/build.log 2>&1 || exit $?
step pytest
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || exit $?
step dist
bash scripts/gpu_dist_rehearsal.sh || exit $?
step bench_all
PROFILE=1 bash scripts/gpu_bench_all.sh || exit $?
step prof_small
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_small -o small -- \
  python bench.py --steps 100 --warmup 20 > gpurun_out/prof_small.log 2>&1 || exit $?
step done
