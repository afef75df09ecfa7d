#!/bin/bash
# One GPU-box pass (run through gpurun): parity tests, rocprof kernel-trace + HBM
# PMC passes of the default bench workload, then the bench line itself (which reads
# the PMC summary this same call produced).  Every GPU step has its own time limit
# and the steps stop at the first failure.
# usage: tools/gpu_round.sh TAG [bench.py args...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || exit $?
bash "$R/tools/rocprof_bench.sh" "gpurun_out/$TAG/prof" --steps 3 --warmup 1 "$@" || exit $?
cp "$O/prof/pmc_traffic.json" "$R/profiles/latest_pmc.json" || exit $?
cd "$R"
timeout -k 10 900 python -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.log" || exit $?
cat "$O/bench.json"
