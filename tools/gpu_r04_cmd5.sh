#!/bin/bash
# r04: parity subset on the current build, then env A/Bs (one process) and
# build-time A/Bs (a process per setting)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batches.py tests/test_gpu_configs.py \
    tests/test_gpu_reference_cases.py tests/test_gpu_sim_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/r04t5.log 2>&1 || { tail -30 gpurun_out/r04t5.log; exit 1; }
tail -1 gpurun_out/r04t5.log
bash tools/gpu_ab_env.sh r04ab5 "" - base= seg64=CHR_TAIL_LONE:0 shp1=CHR_SHADE_PREFETCH2:0 dl0=CHR_TRACE_DRAIN_LONE:0 || exit 1
bash tools/gpu_ab_procs.sh r04bvh5 2 "--steps 20 --warmup 5" base= sweep64=CHR_WIDE_SWEEP:64 leaf3=CHR_WIDE_LEAF_MAX:3 \
    leaf3s=CHR_WIDE_LEAF_MAX:3,CHR_WIDE_SWEEP:64
