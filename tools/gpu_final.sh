#!/bin/bash
# Round-end GPU pass (run through gpurun): smoke(), the GPU test suite, the
# rocprof kernel-trace + HBM PMC passes of the driver's bench command, then the
# bench line itself (reading the PMC summary this same call produced).
# usage (GPU box): tools/gpu_final.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -20 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
if [ "${WITH_PROF:-1}" = 1 ]; then
  bash "$R/tools/rocprof_bench.sh" "gpurun_out/$TAG/prof" --steps 20 --warmup 5 || exit $?
  cp "$O/prof/pmc_traffic.json" "$R/profiles/latest_pmc.json" || exit $?
fi
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 "$R/bench.py" --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log" || exit $?
cut -c1-300 "$O/bench.json"
