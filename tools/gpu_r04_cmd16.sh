#!/bin/bash
# r04: finer Morton direction cells for the binned first step: 10+10 / 11+11 / 12+12 bits
# (CHR_BIN_KEY=2/3/4) against row-major 8+8
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab16 "CHR_BIN_KEY=4" "tests/test_gpu_batches.py tests/test_gpu_configs.py" \
    base= k2=CHR_BIN_KEY:2 k3=CHR_BIN_KEY:3 k4=CHR_BIN_KEY:4
