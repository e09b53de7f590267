#!/bin/bash
# xGMI all-reduce local-cost figures on a 1-GPU box: kernel us / GB/s per bucket size and form,
# grid-cap and coarse-grained-buffer A/B, world 4, and 2-rank bench.py runs (allreduce_us per model).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/xgmi
mkdir -p $OUT
fatal() { case "$1" in 0) return 0;; *) echo "FATAL rc=$1 at $2" | tee -a $OUT/status.log; exit "$1";; esac; }
for v in "X=1"; do
  env $v timeout -k 10 300 python scripts/xgmi_local_bench.py --world 2 >> $OUT/local.jsonl 2>> $OUT/local.err; fatal $? "$v"
done
timeout -k 10 300 python scripts/xgmi_local_bench.py --world 4 >> $OUT/local.jsonl 2>> $OUT/local.err; fatal $? world4
export MTA_DIST_BACKEND=gloo MTA_ALLREDUCE=xgmi
for m in "small fast 1" "mlp_small gpu_fast 1" "mlp_large gpu_fast 64" "transformer_encoder gpu_fast 1"; do
  set -- $m
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29700 + RANDOM % 200)) bench.py --gpus 2 --steps 40 --warmup 10 --model $1 --trainer $2 \
    --batch $3 >> $OUT/bench2.jsonl 2>> $OUT/bench2.err; fatal $? "bench $1"
done
echo done >> $OUT/status.log
