#!/bin/bash
# LSTM defaults DX_DELAY 4 + PRIO 1: LSTM GPU tests, headline x3, medium / large / B=64 benches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu -k "lstm or stack or engine or smoke or fused" -x > $O/pytest.log 2>&1 || exit $?
for i in 1 2 3; do
  timeout -k 10 300 python bench.py >> $O/bench_headline.jsonl 2>> $O/bench.err || exit $?
done
for m in medium large; do
  timeout -k 10 300 python bench.py --model $m --steps 100 --warmup 10 >> $O/bench_lstm.jsonl 2>> $O/bench.err || exit $?
done
timeout -k 10 300 python bench.py --batch 64 --steps 100 --warmup 10 >> $O/bench_lstm.jsonl 2>> $O/bench.err || exit $?
