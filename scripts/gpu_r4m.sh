#!/bin/bash
# LSTM stack knob A/B on the headline shape (N=100 L=2 prec=3 T=60): base, static priority, helper-wave delays
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4m2
mkdir -p $O
for round in 1 2; do
  for b in stk_base stk_d4 stk_d6 stk_d8 stk_d12 stk_d4p1 stk_d8p1 stk_p1; do
    echo "## $b round $round" >> $O/knobs.txt
    timeout -k 10 90 ./tools_bin/$b 100 2 3 60 0 >> $O/knobs.txt 2>&1 || exit $?
  done
done
