#!/bin/bash
# Per-host-step survivor counts and walk-cost histograms (usage: tools/gpu_r02_steps.sh TAG):
# one bench propagate with CHR_TRACE_STEPS=1, default variant then the counting variant (5).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-steps}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd /tmp && export TMPDIR=/tmp
CHR_TRACE_STEPS=1 timeout -k 10 400 python3 "$R/bench.py" --steps 2 --warmup 0 --no-cpu-baseline --no-count \
    > "$O/bench_default.json" 2> "$O/steps_default.log" || { echo "default rc=$?"; exit 1; }
CHR_TRACE_STEPS=1 CHR_PROPAGATE_VARIANT=5 timeout -k 10 400 python3 "$R/bench.py" --steps 1 --warmup 0 \
    --no-cpu-baseline --no-count > "$O/bench_count.json" 2> "$O/steps_count.log" || { echo "count rc=$?"; exit 1; }
grep -c "alive" "$O/steps_default.log"
