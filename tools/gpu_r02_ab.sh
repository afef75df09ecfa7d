#!/bin/bash
# Same-box A/B of two in-tree builds (usage: tools/gpu_r02_ab.sh TAG [TESTS]):
# optional GPU parity tests of the default library, then the driver's bench
# command with the default library (new) and with libchroma_amd_ab.so (old),
# each run twice, interleaved.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-ab}
TESTS=${2:-}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
if [ -n "$TESTS" ]; then
    timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1
    rc=$?
    tail -3 "$O/pytest_gpu.log"
    [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
    timeout -k 10 300 python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-count \
        > "$O/new_$i.json" 2> "$O/new_$i.log" || { echo "new $i failed"; exit 1; }
    CHROMA_AMD_LIB=$R/chroma-lite_amd/chroma/_lib/libchroma_amd_ab.so timeout -k 10 300 python3 "$R/bench.py" \
        --steps 20 --warmup 5 --no-cpu-baseline --no-count > "$O/old_$i.json" 2> "$O/old_$i.log" \
        || { echo "old $i failed"; exit 1; }
    python3 -c "
import json
for t in ('new_$i', 'old_$i'):
    d = json.load(open('$O/' + t + '.json'))
    print(t, round(d['value'] / 1e6, 1), 'M/s', round(d['ms_per_step'], 2), 'ms/step trace',
          round(d['detail']['trace_ms_per_step'], 2), 'ms')"
done
