#!/bin/bash
# The batches' ncopies / use_weights test, then the bench lines of the other
# BASELINE configs (C2 tiny 1M, C3 demo.detector() 10M, C5 scintillator 10M).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02_configs
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_batches.py -k copies -x -v --timeout 200 --timeout-method thread \
    > "$O/pytest_batches_copies.log" 2>&1 || { tail -20 "$O/pytest_batches_copies.log"; exit 1; }
tail -2 "$O/pytest_batches_copies.log"
bash "$R/tools/bench_configs.sh" gpurun_out/r02_configs || exit $?
for f in "$O"/bench_*.json; do echo "$f"; cut -c1-150 "$f"; done
