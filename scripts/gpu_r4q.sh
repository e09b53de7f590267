#!/bin/bash
# zero-padded dh from the one-launch decoder (MLP encoder reads it in place): tests + mlp_small benches + trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu -k "fused or extras or loss or decoder or heads" > $O/pytest.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --model mlp_small --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_ms.jsonl 2>> $O/bench.err || exit $?
  timeout -k 10 300 python bench.py --model mlp_small --trainer fast --steps 200 --warmup 20 >> $O/bench_msf.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ms -- python bench.py --model mlp_small --trainer gpu_fast --steps 100 --warmup 20 > $O/prof.log 2>&1 || exit $?
