#!/bin/bash
# Bench lines after the batch-pool change: the default command (3 steps, 1
# warm-up), the driver's command, then the other BASELINE configs.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02_configs2
mkdir -p "$O"
cd "$R"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 500 python -u bench.py > "$O/bench_29k_default.json" 2> "$O/bench_29k_default.log" || exit $?
cut -c1-200 "$O/bench_29k_default.json"
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-count > "$O/bench_29k_20_5.json" 2> "$O/bench_29k_20_5.log" || exit $?
cut -c1-200 "$O/bench_29k_20_5.json"
bash "$R/tools/bench_configs.sh" gpurun_out/r02_configs2 || exit $?
for f in "$O"/bench_*.json; do echo "$f"; cut -c1-200 "$f"; done
