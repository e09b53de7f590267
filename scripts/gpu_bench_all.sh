#!/bin/bash
# 1-GPU throughput of every model family, trial packing (--concurrent k), optional rocprof
# kernel traces (PROFILE=1) and PMC counter passes over the extras' GEMM / norm / attention kernels (PMC=1).
# The extras run under trainer=gpu_fast (bf16-mixed: BASELINE.json configs 2-4 name bf16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${OUT:-bench_all}
mkdir -p $OUT
J=$OUT/bench_all.jsonl
: > $J
export TMPDIR=/tmp
run() {
  echo "[bench_all] $*" >&2
  timeout -k 10 400 python bench.py --steps ${STEPS:-100} --warmup 10 "$@" >> $J 2>> $OUT/bench_all.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc: $*" >> $OUT/bench_all.err; exit $rc; fi
}
if [ -z "$SKIP_MODELS" ]; then
run --model small --loss mse
run --model small --loss nll
run --model small --loss combined
run --model medium --loss mse
run --model large --loss mse
run --model small --loss mse --batch 8
run --model small --loss mse --batch 64
run --model mlp_small --loss mse --trainer gpu_fast
run --model mlp_large --loss mse --batch 64 --trainer gpu_fast
run --model mlp_small --loss mse --trainer fast
run --model transformer_encoder --loss mse --trainer gpu_fast
run --model transformer_encoder --loss combined --batch 8 --trainer gpu_fast
fi
if [ -n "$CONCURRENT" ]; then
  for k in 2 4 8; do run --model small --loss mse --concurrent $k --steps 400; done
fi
if [ -n "$PROFILE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_tr -o tr -- python bench.py --model transformer_encoder --trainer gpu_fast --steps 50 --warmup 10 > $OUT/prof_tr.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_mlp -o mlp -- python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 50 --warmup 10 > $OUT/prof_mlp.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_small -o small -- python bench.py --steps 100 --warmup 20 > $OUT/prof_small.log 2>&1 || exit $?
fi
if [ -n "$PMC" ]; then
  P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
  P2="SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum GRBM_COUNT"
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_mlp$i -o pmc -- python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 8 --warmup 2 > $OUT/pmc_mlp$i.log 2>&1 || exit $?
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_tr$i -o pmc -- python bench.py --model transformer_encoder --trainer gpu_fast --steps 8 --warmup 2 > $OUT/pmc_tr$i.log 2>&1 || exit $?
  done
fi
if [ -n "$GEMM_PMC" ]; then
  # the 256 x 256 GEMM (tools_bin/gemm_probe, scripts/build_probes.sh gemm) at 4096^3 and the mlp_large shapes
  G1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
  G2="TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_COUNT"
  i=0
  for P in "$G1" "$G2"; do
    i=$((i+1))
    for sh in "4096 4096 4096 0" "6400 2048 2048 0 1" "6400 2048 2048 1" "2048 2048 6400 2"; do
      tag=$(echo $sh | tr ' ' '_')
      timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc_gemm${i}_$tag -o pmc -- ./tools_bin/gemm_probe $sh > $OUT/pmc_gemm${i}_$tag.log 2>&1 || exit $?
    done
  done
fi
echo done >> $OUT/bench_all.err
