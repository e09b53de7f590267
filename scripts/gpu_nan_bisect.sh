#!/bin/bash
# Bisection of the 4-rank graphed bf16 transformer NaN (profiles/r3_s3_dist_rehearsal.txt): 4 gloo ranks share
# cuda:0, MTA_DEBUG_FINITE=1 names the first parameter whose local gradient / value goes non-finite, per variant.
# Usage: scripts/gpu_nan_bisect.sh [variant ...]   (default: all)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/nan
export MTA_DIST_BACKEND=gloo MTA_DEBUG_FINITE=1
RANKS=${RANKS:-4}
run() {  # name, env..., -- extra bench args
  local name=$1; shift
  local envs=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  [ "$1" = "--" ] && shift
  echo "=== $name (${envs[*]}) $*" | tee -a gpurun_out/nan/summary.txt
  env "${envs[@]}" timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$RANKS" \
    --master-addr 127.0.0.1 --master-port $((29600 + RANDOM % 200)) bench.py --gpus "$RANKS" --steps 30 \
    --warmup 5 --model transformer_encoder --trainer gpu_fast "$@" > "gpurun_out/nan/$name.json" \
    2> "gpurun_out/nan/$name.err"
  local rc=$?
  grep -h "\[finite\]\|nonfinite=" "gpurun_out/nan/$name.err" | tee -a gpurun_out/nan/summary.txt
  echo "rc=$rc" | tee -a gpurun_out/nan/summary.txt
  case $rc in 124|137|134|139) echo "stopping after rc=$rc"; exit $rc;; esac
  return 0
}
VARIANTS=${*:-"default hwq1 noslab nodrop spg1"}
for v in $VARIANTS; do
  case $v in
    default) run default X=1 ;;
    hwq1) run hwq1 GPU_MAX_HW_QUEUES=1 ;;
    noslab) run noslab MTA_GEMM_SLABS=0 ;;
    nodrop) run nodrop X=1 -- --set model.dropout=0 ;;
    spg1) run spg1 X=1 -- --steps-per-graph 1 ;;
    nographs) run nographs X=1 -- --no-graphs ;;
    serial) run serial AMD_SERIALIZE_KERNEL=3 ;;
  esac
done
