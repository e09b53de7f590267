#!/bin/bash
# wgrad split target re-check with every round-4 default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
for w in 128 112 160 144 128; do
  MTA_WGRAD_WGS=$w timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 > $O/tr_$w.json 2>> $O/bench.err || exit $?
  echo "transformer $w $(cat $O/tr_$w.json)" >> $O/sweep.txt
done
