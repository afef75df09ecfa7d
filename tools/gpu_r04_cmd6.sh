#!/bin/bash
# r04: the trace kernel at 5 waves per SIMD (CHR_TRACE_LAYOUT=3) against the default,
# parity tests of the new layout first
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab6 "CHR_TRACE_LAYOUT=3" "tests/test_gpu_batches.py tests/test_gpu_configs.py" \
    base= lay3=CHR_TRACE_LAYOUT:3 lay3d2=CHR_TRACE_LAYOUT:3,CHR_TRACE_DRAIN:2
