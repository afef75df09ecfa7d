#!/bin/bash
# r04: shade SC (prefetch waited for before the write-back; default) against CHR_SHADE_SC=0,
# plus the same pair with every slot event recorded (kernel ms per step)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_ab_env.sh r04ab10 "" "tests/test_gpu_batches.py tests/test_gpu_parity.py" \
    base= sc0=CHR_SHADE_SC:0 base_t=CHR_SLOT_TIMING:1 sc0_t=CHR_SHADE_SC:0,CHR_SLOT_TIMING:1
