#!/bin/bash
# Tail-kernel check (usage: tools/gpu_r02_tail.sh TAG): GPU tests, then the
# driver's bench command with the wave-adaptive tail (default) and with the
# fixed 8-lane group tail (CHR_TAIL=group) for the A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-tail}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -4 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench_wave.json" 2> "$O/bench_wave.log"
rc=$?
echo "bench wave rc=$rc"; cut -c1-200 "$O/bench_wave.json"
[ $rc -eq 0 ] || exit $rc
CHR_TAIL=group timeout -k 10 400 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
    > "$O/bench_group.json" 2> "$O/bench_group.log"
rc=$?
echo "bench group rc=$rc"; cut -c1-200 "$O/bench_group.json"
exit $rc
