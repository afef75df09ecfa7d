#!/bin/bash
# r04: trace kernel node step with derived child offsets (CHR_TRACE_LAYOUT=4, five node
# loads) against the default, parity tests of the variant first
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab7 "CHR_TRACE_LAYOUT=4" "tests/test_gpu_batches.py tests/test_gpu_configs.py" \
    base= doff=CHR_TRACE_LAYOUT:4
