#!/bin/bash
# r5v: PMC passes over the 256x256 GEMM forms on 4096^3 and the mlp_large forward (effective clock, MFMA busy, LDS, L2)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5v
mkdir -p $O
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_COUNT"
for v in -1 1; do
  for sh in "sq 4096" "mlp_large fwd"; do
    tag="v${v}_$(echo $sh | tr ' ' '_')"
    timeout -s KILL 90 rocprofv3 --pmc $P1 --output-format csv -d $O/$tag/p1 -o p -- python scripts/gemm_bench.py --only "$sh" --variants=$v --no-blas > $O/$tag.p1.log 2>&1 || { echo "p1 $tag rc=$?" >> $O/status.log; exit 1; }
    timeout -s KILL 90 rocprofv3 --pmc $P2 --output-format csv -d $O/$tag/p2 -o p -- python scripts/gemm_bench.py --only "$sh" --variants=$v --no-blas > $O/$tag.p2.log 2>&1 || { echo "p2 $tag rc=$?" >> $O/status.log; exit 1; }
  done
done
echo done >> $O/status.log
