#!/bin/bash
# weight-gradient split target A/B (MTA_WGRAD_WGS) on the transformer and mlp_small
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4k2
mkdir -p $O
for w in 128 64 96 32 128 256; do
  MTA_WGRAD_WGS=$w timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 > $O/tr_$w.json 2>> $O/bench.err || exit $?
  echo "transformer $w $(cat $O/tr_$w.json)" >> $O/sweep.txt
done
for w in 256 128 64 256; do
  MTA_WGRAD_WGS=$w timeout -k 10 300 python bench.py --model mlp_small --trainer gpu_fast --steps 200 --warmup 20 > $O/ms_$w.json 2>> $O/bench.err || exit $?
  echo "mlp_small $w $(cat $O/ms_$w.json)" >> $O/sweep.txt
done
for w in 256 128 256; do
  MTA_WGRAD_WGS=$w timeout -k 10 300 python bench.py --model transformer_encoder --loss combined --batch 8 --trainer gpu_fast --steps 50 --warmup 10 > $O/trb8_$w.json 2>> $O/bench.err || exit $?
  echo "transformer_b8 $w $(cat $O/trb8_$w.json)" >> $O/sweep.txt
done
