#!/bin/bash
# trial packing: k independent B=1 headline trainers on one GPU, k = 2..8 (where the k=4 -> 8 drop starts)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pack
mkdir -p $O
for k in 2 3 4 5 6 7 8; do
  echo "k=$k $(date +%T)" >> $O/progress.log
  timeout -k 10 240 python bench.py --concurrent $k --steps 400 --warmup 20 >> $O/pack.jsonl 2>> $O/pack.err || exit $?
done
