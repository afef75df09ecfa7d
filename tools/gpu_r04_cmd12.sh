#!/bin/bash
# r04: trace_kernel refill threshold R (48 default; 56, 64) and node / triangle step
# threshold F (6 default; 5, 7)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab12 "CHR_TRACE_R=64" "tests/test_gpu_batches.py" \
    base= r56=CHR_TRACE_R:56 r64=CHR_TRACE_R:64 f5=CHR_TRACE_F:5 f7=CHR_TRACE_F:7
