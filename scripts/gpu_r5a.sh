#!/bin/bash
# r5 first session: smoke (two precisions), the new launcher / graph-audit / step-1 gradient tests, headline bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_graphs.py \
  tests/test_gpu_launch.py "tests/test_gpu_dist_trainer.py::test_step1_summed_gradient_matches_global_batch" \
  "tests/test_gpu_extras.py::test_mlp_grad_producers_match_accumulating_path" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/headline.json 2> $O/headline.err || exit $?
