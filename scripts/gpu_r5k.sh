#!/bin/bash
# thesis accuracy: two more seeds at the default precision (sign-basin statistics of the NLL / combined losses)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_thesis.sh 100 high "2 3"
