#!/bin/bash
# PMC passes of the default bench workload (usage: tools/gpu_r02_pmc.sh TAG "COUNTERS" ["COUNTERS" ...]):
# one rocprofv3 --pmc run per counter set (the guide's per-block limits apply to
# each set), bench.py --steps 3 --warmup 1 --no-count --no-cpu-baseline.
# Also writes the counter list of this box (rocprofv3 -L) once.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1
shift
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd /tmp && export TMPDIR=/tmp
[ -f "$O/avail.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$O/avail.txt" 2>&1 || true
i=0
for C in "$@"; do
    i=$((i + 1))
    echo "pass $i: $C"
    timeout -s KILL 500 rocprofv3 --pmc $C --output-format csv -d "$O/pmc$i" -o run -- \
        python3 "$R/bench.py" --steps 3 --warmup 1 --no-count --no-cpu-baseline \
        > "$O/pmc$i.json" 2> "$O/pmc$i.log" || { echo "pass $i rc=$?"; tail -5 "$O/pmc$i.log"; exit 1; }
done
echo "pmc ok"
