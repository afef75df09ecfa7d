#!/bin/bash
# r04: walk-order carry (later steps walk in the previous step's walk order, CHR_WALK_CARRY=1)
# on top of the finer first-step binning
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab17 "CHR_WALK_CARRY=1" "tests/test_gpu_batches.py" \
    base= carry=CHR_WALK_CARRY:1
