#!/bin/bash
# 1-GPU throughput of every model family; optional rocprof of the extras (PROFILE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/bench_all.jsonl
: > $OUT
run() {
  echo "[bench_all] $*" >&2
  timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 10 "$@" >> $OUT 2>> gpurun_out/bench_all.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >> gpurun_out/bench_all.err; exit $rc; fi
}
run --model small --loss mse
run --model small --loss combined
run --model medium --loss mse
run --model large --loss mse
run --model small --loss mse --batch 8
run --model small --loss mse --batch 64
run --model mlp_small --loss mse
run --model mlp_large --loss mse --batch 64
run --model transformer_encoder --loss mse
run --model transformer_encoder --loss combined --batch 8
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tr -o tr -- python bench.py --model transformer_encoder --steps 50 --warmup 10 > gpurun_out/prof_tr.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlp -o mlp -- python bench.py --model mlp_large --batch 64 --steps 50 --warmup 10 > gpurun_out/prof_mlp.log 2>&1 || exit $?
fi
echo done >> gpurun_out/bench_all.err
