#!/bin/bash
# producers test (relaxed to the atomic-order noise floor) + the whole GPU suite, mlp_large producers A/B + trace,
# kernel-level timing of the wgrad split sweep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
{ timeout -k 10 60 ./tools_bin/ffn_probe_0 && timeout -k 10 60 ./tools_bin/ffn_probe_1 && timeout -k 10 60 ./tools_bin/ffn_probe_1 6240 0; } > $O/ffn_probe.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for f in 1 0 1 0; do
  MTA_OPTIM_PRODUCERS=$f timeout -k 10 300 python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 100 --warmup 10 >> $O/bench_mlp.jsonl 2>> $O/bench.err || exit $?
done
MTA_OPTIM_PRODUCERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 92 --warmup 10 > $O/prof_mlp.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_sweep -o sweep -- python scripts/wgrad_split_sweep.py > $O/prof_sweep.log 2>&1 || exit $?
