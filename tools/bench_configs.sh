#!/bin/bash
# Bench lines for the other BASELINE.json configs on one GPU (run through gpurun):
#   C2 tiny detector 1M photons, C3 demo.detector() 10M photons, C5 scintillator detector 10M photons.
# usage: tools/bench_configs.sh OUTDIR
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/$1
mkdir -p "$O"
cd "$R"
timeout -k 10 400 python -u bench.py --detector tiny --photons 1000000 --steps 20 --warmup 5 > "$O/bench_tiny_1M.json" 2> "$O/bench_tiny_1M.log" || exit $?
timeout -k 10 600 python -u bench.py --detector demo --photons 10000000 --steps 20 --warmup 5 > "$O/bench_demo_10M.json" 2> "$O/bench_demo_10M.log" || exit $?
timeout -k 10 600 python -u bench.py --detector scint --photons 10000000 --steps 20 --warmup 5 > "$O/bench_scint_10M.json" 2> "$O/bench_scint_10M.log" || exit $?
