#!/bin/bash
# r04: trace_kernel with prefetched ray records (CHR_TRACE_PF=R) against the default refill;
# parity tests under PF first
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab11 "CHR_TRACE_PF=32" "tests/test_gpu_batches.py tests/test_gpu_configs.py tests/test_gpu_parity.py" \
    base= pf48=CHR_TRACE_PF:48 pf32=CHR_TRACE_PF:32 pf16=CHR_TRACE_PF:16
