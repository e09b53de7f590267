#!/bin/bash
# One parametrised GPU session: runs a PLAN of steps in order, each under its own time limit, and stops at the first
# failing step (no further GPU work after a fault, an abort or a timeout).  Replaces the per-session gpu_r5*.sh scripts
# (their evidence is in profiles/ and in git history).
#
#   OUT=<subdir of gpurun_out> PLAN='<step>;<step>;...' bash scripts/gpu_run.sh
#   OUT=... bash scripts/gpu_run.sh plan.txt          (one step per line, '#' comments)
#
# steps (arguments after the keyword are passed through; leading KEY=VALUE tokens set that step's environment):
#   pytest <pytest args>            python -m pytest ... -x -v --timeout 120 --timeout-method thread  -> pytest.log
#   bench <bench.py args>           one JSON line appended to bench.jsonl
#   prof <tag> <bench.py args>      rocprofv3 --kernel-trace --stats of a bench run -> <tag>/
#   pmc <tag> <counters> -- <cmd>   one rocprofv3 --pmc pass (its own run, no trace domains) -> <tag>/
#   probe <N L prec T mode [layer]> tools_bin/stack_s0 + stack_s1 (scripts/build_probes.sh) -> probe.txt
#   tl <N L prec T mode>            tools_bin/stack_tl timeline build (scripts/build_probes.sh) -> probe.txt
#   bin <name> <args>               any tools_bin/<name> (diagnostic variants) -> probe.txt
#   py <script> <args>              python -u <script> <args> -> py.log
#   smoke                           __graft_entry__.smoke() -> smoke.log
# STEP_TIMEOUT (s, default 300) bounds every step; PMC passes are killed at 90 s (an over-subscribed counter block
# hangs rocprofv3 after its "error code 38" line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-run}
mkdir -p "$O"
TO=${STEP_TIMEOUT:-300}
st() { echo "[$(date +%T)] $*" | tee -a "$O/status.log"; }
if [ -n "$1" ]; then mapfile -t STEPS < <(grep -v '^\s*#' "$1" | grep -v '^\s*$'); else IFS=';' read -ra STEPS <<< "${PLAN:-}"; fi
n=0
for s in "${STEPS[@]}"; do
  n=$((n + 1))
  read -ra a <<< "$s"
  # leading KEY=VALUE tokens set the environment of this step only
  envs=()
  while [[ ${a[0]} =~ ^[A-Z_][A-Z0-9_]*= ]]; do envs+=("${a[0]}"); a=("${a[@]:1}"); done
  kind=${a[0]}
  args=("${a[@]:1}")
  for e in "${envs[@]}"; do export "$e"; done
  TO=${STEP_TIMEOUT:-300}  # (a step's own STEP_TIMEOUT=... token applies to that step)
  st "step $n: $s"
  case "$kind" in
    pytest) timeout -k 10 "$TO" python -u -m pytest -x -v --timeout 300 --timeout-method thread "${args[@]}" >> "$O/pytest.log" 2>&1 ;;
    bench) timeout -k 10 "$TO" python bench.py "${args[@]}" >> "$O/bench.jsonl" 2>> "$O/bench.err" ;;
    prof) tag=${args[0]}
          timeout -k 10 "$TO" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/$tag" -o "$tag" -- \
            python bench.py "${args[@]:1}" > "$O/$tag.log" 2>&1 ;;
    pmc) tag=${args[0]}; rest=("${args[@]:1}"); ctr=(); i=0
         while [ $i -lt ${#rest[@]} ] && [ "${rest[$i]}" != "--" ]; do ctr+=("${rest[$i]}"); i=$((i + 1)); done
         timeout -s KILL 90 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d "$O/$tag" -o "$tag" -- \
           "${rest[@]:$((i + 1))}" > "$O/$tag.log" 2>&1 ;;
    probe) prc=0
           for b in stack_s0 stack_s1; do
             timeout -k 10 90 "./tools_bin/$b" "${args[@]}" >> "$O/probe.txt" 2>&1 || { prc=$?; break; }
           done
           (exit $prc) ;;
    tl) timeout -k 10 90 ./tools_bin/stack_tl "${args[@]}" >> "$O/probe.txt" 2>&1 ;;
    bin) b=${args[0]}; echo "== $b ${args[*]:1}" >> "$O/probe.txt"
         timeout -k 10 90 "./tools_bin/$b" "${args[@]:1}" >> "$O/probe.txt" 2>&1 ;;
    py) timeout -k 10 "$TO" python -u "${args[@]}" >> "$O/py.log" 2>&1 ;;
    smoke) timeout -k 10 "$TO" python -u -c "import __graft_entry__ as g; g.smoke()" >> "$O/smoke.log" 2>&1 ;;
    *) st "unknown step kind: $kind"; exit 2 ;;
  esac
  rc=$?
  for e in "${envs[@]}"; do unset "${e%%=*}"; done
  st "step $n rc=$rc"
  if [ $rc -ne 0 ]; then st "FATAL at step $n"; exit $rc; fi
done
st done
