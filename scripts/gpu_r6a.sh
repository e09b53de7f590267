cd "${GRAFT_REPO_ROOT}"
OUT=r6a SPECS="100 2 3 60 0 1;100 4 3 60 0 3;100 8 3 60 0 7;100 8 3 60 0 1" BENCH=1 BENCH_BATCHES=1 bash scripts/gpu_probe.sh && \
for m in medium large; do timeout -k 10 180 python bench.py --steps 200 --warmup 20 --model $m >> gpurun_out/r6a/bench.jsonl 2>>gpurun_out/r6a/bench.err || exit 1; done
