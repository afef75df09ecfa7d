#!/bin/bash
# Check of HEAD on the GPU box: smoke(), the whole GPU suite, the driver's bench
# command (cold node-local cache: flatten + reference BVH + traversal BVH built
# and cached), then a short bench from the warm cache (setup phases only).
# usage (GPU box): tools/gpu_check_head.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/${1:-head}
mkdir -p "$O"
cd "$R"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -20 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 "$R/bench.py" --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log" || exit $?
cut -c1-200 "$O/bench.json"
if [ "${WARM:-1}" = 1 ]; then
  timeout -k 10 300 python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --sequential-steps 0 \
    --timing-steps 0 --no-count > "$O/bench_warm.json" 2> "$O/bench_warm.log" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('warm setup', d['detail']['ranks'][0]['setup'])" "$O/bench_warm.json"
fi
