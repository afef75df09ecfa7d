#!/bin/bash
# r04: the binned first launch's refill threshold alone (CHR_TRACE_R_FIRST=32/56/64; others 48)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab19 "CHR_TRACE_R_FIRST=64" "tests/test_gpu_batches.py" \
    base= rf32=CHR_TRACE_R_FIRST:32 rf56=CHR_TRACE_R_FIRST:56 rf64=CHR_TRACE_R_FIRST:64
