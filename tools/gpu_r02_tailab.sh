#!/bin/bash
# Tail-kernel A/B (usage: tools/gpu_r02_tailab.sh TAG): GPU parity tests of the
# propagate path, then the driver's bench command per tail variant.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-tailab}
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_reference_cases.py \
    -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?
tail -3 "$O/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in 4 3; do
    CHR_TAIL_WAVES=$v timeout -k 10 400 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
        > "$O/bench_w$v.json" 2> "$O/bench_w$v.log"
    rc=$?
    echo "bench waves $v rc=$rc"; cut -c1-160 "$O/bench_w$v.json"
    [ $rc -eq 0 ] || exit $rc
done
