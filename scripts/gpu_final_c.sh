#!/bin/bash
# final evidence with every round-4 default: headline x3 + kernel trace, transformer / mlp_large / mlp_small benches + traces
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final_c
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py >> $O/bench_headline.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_models.jsonl 2>> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 100 --warmup 10 >> $O/bench_models.jsonl 2>> $O/bench.err || exit $?
timeout -k 10 300 python bench.py --model mlp_small --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_models.jsonl 2>> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_small -o small -- python bench.py --steps 100 --warmup 20 > $O/prof_small.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tr -o tr -- python bench.py --model transformer_encoder --trainer gpu_fast --steps 50 --warmup 10 > $O/prof_tr.log 2>&1 || exit $?
