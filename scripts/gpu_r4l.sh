#!/bin/bash
# split-K workgroup target of the 256x256 kernel's accumulating form (MTA_BIG_WGS) on mlp_large B=64
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
for w in 256 128 192 384 512 256 128; do
  MTA_BIG_WGS=$w timeout -k 10 300 python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 100 --warmup 10 > $O/ml_$w.json 2>> $O/bench.err || exit $?
  echo "mlp_large $w $(cat $O/ml_$w.json)" >> $O/sweep.txt
done
