#!/bin/bash
# r5x: FFN forward, one row tile per workgroup vs two per workgroup (the second from a warm instruction cache)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r5x
mkdir -p $O
for M in 6240 12480 49920; do
  for b in ffn_probe ffn_probe_loop; do
    echo -n "$b M=$M :: " >> $O/ffn_loop.log
    timeout -k 5 60 probe_bin/$b $M 2>&1 | grep "fwd" | head -1 >> $O/ffn_loop.log || exit 1
  done
done
echo done >> $O/ffn_loop.log
