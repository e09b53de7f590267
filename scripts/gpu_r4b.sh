#!/bin/bash
# extras + optimizer tests, transformer (fused halves on / off) and mlp_large (gradient producers on / off) benches,
# kernel traces of both
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 200 python -u scripts/debug_producers.py > $O/debug_producers.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_extras.py tests/test_gpu_kernels.py -k "not grad_producers" > $O/pytest.log 2>&1 || exit $?
# (ffn, attn, wgrad-nn): all fused, no NN wgrads, FFN only, unfused
for v in 111 110 100 000; do
  MTA_TR_FFN=${v:0:1} MTA_TR_ATTN=${v:1:1} MTA_TR_WGRAD_NN=${v:2:1} timeout -k 10 300 python bench.py --model transformer_encoder --trainer gpu_fast --steps 200 --warmup 20 >> $O/bench_tr.jsonl 2>> $O/bench.err || exit $?
done
for f in 1 0 1 0; do
  MTA_OPTIM_PRODUCERS=$f timeout -k 10 300 python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 100 --warmup 10 >> $O/bench_mlp.jsonl 2>> $O/bench.err || exit $?
done
MTA_TR_ATTN=1 MTA_TR_WGRAD_NN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_tr -o tr -- python bench.py --model transformer_encoder --trainer gpu_fast --steps 92 --warmup 10 > $O/prof_tr.log 2>&1 || exit $?
MTA_OPTIM_PRODUCERS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o mlp -- python bench.py --model mlp_large --trainer gpu_fast --batch 64 --steps 92 --warmup 10 > $O/prof_mlp.log 2>&1 || exit $?
