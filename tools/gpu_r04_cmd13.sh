#!/bin/bash
# r04: 2-triangle leaves aligned to one line (CHR_WIDE_ALIGN2=1, build-time) against the
# default layout; wide-BVH / walker parity tests under it first
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
mkdir -p gpurun_out/r04bvh13
CHR_WIDE_ALIGN2=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/r04bvh13/pytest.log 2>&1 || { tail -30 gpurun_out/r04bvh13/pytest.log; exit 1; }
tail -1 gpurun_out/r04bvh13/pytest.log
bash tools/gpu_ab_procs.sh r04bvh13 2 "--steps 20 --warmup 5" base= align2=CHR_WIDE_ALIGN2:1
