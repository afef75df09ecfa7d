#!/bin/bash
# r04: shade kernel with static memory-op counts (peeled first iteration, prefetch and
# write-back outside branches; default) against the r04 shade (CHR_SHADE_SC=0)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab9 "" "tests/test_gpu_batches.py tests/test_gpu_configs.py tests/test_gpu_parity.py" \
    base= sc0=CHR_SHADE_SC:0
