#!/bin/bash
# GPU check (round 2): the driver's bench command under rocprofv3 kernel trace,
# then the GPU test suite.  usage (GPU box): tools/gpu_r02_check.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-check}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
    python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log"
rc=$?
echo "bench rc=$rc"; cut -c1-300 "$O/bench.json"
[ $rc -eq 0 ] || { tail -20 "$O/bench.log"; exit $rc; }
cd "$R"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -15 "$O/pytest_gpu.log"
exit $rc
