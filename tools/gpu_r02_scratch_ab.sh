#!/bin/bash
# Round-2 GPU check: the driver's exact bench command (--steps 20 --warmup 5)
# under rocprofv3 --kernel-trace --stats, with this tree's library (no scratch
# in the default kernels) and with the round-1 library (trace_kernel with a
# 944 B/lane private stack), same box, so the round-1 43x gap is explained by
# measurement.  usage (GPU box): tools/gpu_r02_scratch_ab.sh
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r02
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_new" -o run -- \
    python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench_new.json" 2> "$O/bench_new.log" \
    || { echo "new bench failed"; tail -20 "$O/bench_new.log"; exit 2; }
echo "new library:"; cut -c1-400 "$O/bench_new.json"
CHROMA_AMD_LIB=$R/chroma-lite_amd/chroma/_lib/libchroma_amd_r01.so timeout -k 10 480 \
    rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_old" -o run -- \
    python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-count --no-cpu-baseline \
    > "$O/bench_old.json" 2> "$O/bench_old.log" || { echo "old bench failed"; tail -20 "$O/bench_old.log"; exit 3; }
echo "round-1 library:"; cut -c1-400 "$O/bench_old.json"
