#!/bin/bash
# GPU check (round 2, session 3): the batches parity tests, then the driver's
# bench command (pipelined steps) and the same with --no-pipeline.
# usage (GPU box): tools/gpu_s3_pipe.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-pipe}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_batches.py -x -v --timeout 500 --timeout-method thread \
    > "$O/pytest_batches.log" 2>&1
rc=$?
tail -12 "$O/pytest_batches.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log"
rc=$?
echo "bench rc=$rc"; cut -c1-400 "$O/bench.json"
[ $rc -eq 0 ] || { tail -20 "$O/bench.log"; exit $rc; }
timeout -k 10 400 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-pipeline --no-cpu-baseline --no-count \
    > "$O/bench_nopipe.json" 2> "$O/bench_nopipe.log"
rc=$?
echo "bench nopipe rc=$rc"; cut -c1-300 "$O/bench_nopipe.json"
exit $rc
