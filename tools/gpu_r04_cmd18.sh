#!/bin/bash
# r04: 11+11-bit direction cells in Hilbert order (CHR_BIN_KEY=5) against Morton (default 3)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab18 "CHR_BIN_KEY=5" "tests/test_gpu_batches.py" base= hilbert=CHR_BIN_KEY:5
