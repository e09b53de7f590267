#!/bin/bash
# Round-2 recurrence study: stack-probe timings (drain lag 1 vs 2), s_memtime stamp shares, PMC counter
# passes on the pipelined LSTM kernels, then the product GPU tests.  Any signal / timeout exit ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r2b
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { if [ "$1" -ge 124 ]; then echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1"; fi; }
st() { echo "[$(date +%T)] $*" | tee -a $OUT/status.log; }
for b in stack_s0_l1 stack_s0_l2 stack_s1_l1 stack_s1_l2; do
  for n in 100 800; do
    timeout -k 10 60 ./tools_bin/$b $n 2 >> $OUT/probe.txt 2>&1; rc=$?; st "$b N=$n rc=$rc"; fatal $rc $b
  done
done
timeout -k 10 60 ./tools_bin/stack_s0_l1 100 4 >> $OUT/probe.txt 2>&1; rc=$?; st "L4 lag1 rc=$rc"; fatal $rc l4
timeout -k 10 60 ./tools_bin/stack_s0_l2 100 4 >> $OUT/probe.txt 2>&1; rc=$?; st "L4 lag2 rc=$rc"; fatal $rc l4b
rocprofv3 -L > $OUT/counters_avail.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_INSTS_VALU_MFMA_BF16 SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d $OUT/pmc$i -o pmc -- ./tools_bin/stack_s0_l1 100 2 > $OUT/pmc$i.log 2>&1; rc=$?; st "pmc$i rc=$rc"; fatal $rc pmc$i
done
st pytest
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; st "pytest rc=$rc"; fatal $rc pytest
st done
