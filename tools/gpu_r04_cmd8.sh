#!/bin/bash
# r04: the two-level lone walker (CHR_TAIL_LONE=2): walker parity tests first (short
# limit), then the GPU suite's batch / config tests under it, then the A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r04ab8
timeout -k 10 300 python -u -m pytest tests/test_gpu_batches.py -k "walker or mirror" -m gpu -x -v --timeout 240 \
    --timeout-method thread > gpurun_out/r04ab8/pytest_walkers.log 2>&1 || { tail -30 gpurun_out/r04ab8/pytest_walkers.log; exit 1; }
tail -2 gpurun_out/r04ab8/pytest_walkers.log
bash tools/gpu_ab_env.sh r04ab8 "CHR_TAIL_LONE=2" "tests/test_gpu_batches.py tests/test_gpu_configs.py tests/test_gpu_parity.py" \
    base= lone2=CHR_TAIL_LONE:2
