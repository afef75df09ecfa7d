#!/bin/bash
# Same-box A/B of one library under two environments (usage:
# tools/gpu_r02_envab.sh TAG "ENV_B" [TESTS]): optional GPU tests, then the
# driver's bench command with the default environment (A) and with ENV_B (B),
# interleaved, twice each.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1
ENVB=$2
TESTS=${3:-}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
if [ -n "$TESTS" ]; then
    timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 150 --timeout-method thread \
        > "$O/pytest_gpu.log" 2>&1
    rc=$?
    tail -3 "$O/pytest_gpu.log"
    [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
for i in 1 2; do
    timeout -k 10 300 python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-count \
        > "$O/a_$i.json" 2> "$O/a_$i.log" || { echo "A $i failed"; tail -5 "$O/a_$i.log"; exit 1; }
    env $ENVB timeout -k 10 300 python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-count \
        > "$O/b_$i.json" 2> "$O/b_$i.log" || { echo "B $i failed"; tail -5 "$O/b_$i.log"; exit 1; }
    python3 -c "
import json
for t in ('a_$i', 'b_$i'):
    d = json.load(open('$O/' + t + '.json'))
    print(t, round(d['value'] / 1e6, 1), 'M/s', round(d['ms_per_step'], 2), 'ms/step kernels',
          round(d['detail']['kernel_ms_per_step'], 2), 'trace', round(d['detail']['trace_ms_per_step'], 2),
          'host steps', d['detail']['host_steps_per_propagate'])"
done
