#!/bin/bash
# r04: the binned first step's walk order: direction cells in Morton order (8+8 bits,
# CHR_BIN_KEY=1) and finer 10+10-bit Morton cells (a 20-bit sort, =2) against row-major 8+8
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab15 "CHR_BIN_KEY=2" "tests/test_gpu_batches.py tests/test_gpu_configs.py" \
    base= k1=CHR_BIN_KEY:1 k2=CHR_BIN_KEY:2
