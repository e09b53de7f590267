#!/bin/bash
# One GPU-box session: build check, smoke, GPU tests, 1-GPU bench (+ optional rocprof).
# Every GPU step has its own time limit; any abort/fault/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
stop_if_fatal() {  # $1 = exit code, $2 = step name
  case "$1" in
    0|1) return 0 ;;                       # ok / ordinary test failure
    *) echo "FATAL: step $2 exited $1; stopping" | tee -a $OUT/status.log; exit "$1" ;;
  esac
}
echo "start $(date)" > $OUT/status.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> $OUT/status.log; stop_if_fatal $rc smoke
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $OUT/status.log; stop_if_fatal $rc pytest
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-200} --warmup 20 ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc" >> $OUT/status.log; stop_if_fatal $rc bench
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- \
    python bench.py --steps 100 --warmup 20 ${BENCH_ARGS:-} > $OUT/prof_bench.log 2>&1
  rc=$?; echo "rocprof rc=$rc" >> $OUT/status.log; stop_if_fatal $rc rocprof
fi
echo "done $(date)" >> $OUT/status.log
