#!/bin/bash
# r04: is the ray counter's atomic contended?  Claim-ahead refills (CHR_TRACE_AHEAD=1) with
# chunks of 64 / 128 / 256 indices (a quarter of the atomics at 256) against the default
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab14 "CHR_TRACE_AHEAD=1 CHR_TRACE_CLAIM=256" "tests/test_gpu_batches.py" \
    base= ca64=CHR_TRACE_AHEAD:1 ca128=CHR_TRACE_AHEAD:1,CHR_TRACE_CLAIM:128 ca256=CHR_TRACE_AHEAD:1,CHR_TRACE_CLAIM:256
