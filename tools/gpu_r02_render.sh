#!/bin/bash
# Renderer + tail check (usage: tools/gpu_r02_render.sh TAG): the render GPU
# tests first, then the whole GPU suite, then the driver's bench command.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-render}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_render.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/pytest_render.log" 2>&1
rc=$?
tail -4 "$O/pytest_render.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log"
rc=$?
echo "bench rc=$rc"; cut -c1-200 "$O/bench.json"
exit $rc
