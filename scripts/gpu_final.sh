#!/bin/bash
# closing evidence of a round: whole GPU suite, smoke(), every-model bench with kernel traces (and PMC passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${FINAL_TAG:-final}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/status.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke rc=$?" >> $O/status.log; exit 1; }
echo "smoke ok" >> $O/status.log
OUT=${FINAL_TAG:-final}/bench_all STEPS=200 PROFILE=1 bash scripts/gpu_bench_all.sh || { echo "bench_all rc=$?" >> $O/status.log; exit 1; }
echo done >> $O/status.log
