#!/bin/bash
# Round-2 diagnostics on the GPU box (usage: tools/gpu_r02_diag.sh TAG):
#   1. FETCH_SIZE calibration on gathers of known bytes (tools/gather_calib)
#   2. the driver's bench command (20/5) with the tail-launch diagnostics
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-diag}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/calib_fetch" -o run -- \
    "$R/tools/gather_calib" > "$O/calib.json" 2> "$O/calib.log" || { echo "calib rc=$?"; tail "$O/calib.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/calib_trace" -o run -- \
    "$R/tools/gather_calib" > /dev/null 2>> "$O/calib.log" || { echo "calib trace rc=$?"; exit 1; }
echo "calib ok"
timeout -k 10 600 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$O/bench.json" 2> "$O/bench.log"
rc=$?
echo "bench rc=$rc"; cut -c1-300 "$O/bench.json"
exit $rc
