#!/bin/bash
# Profile the default bench workload with rocprofv3 (run on the GPU box):
#   1. --kernel-trace --stats      -> per-kernel time (profiles/<round>/rocprof_kernel_stats.csv)
#   2. --pmc FETCH_SIZE            -> HBM read bytes per dispatch (own pass)
#   3. --pmc WRITE_SIZE            -> HBM write bytes per dispatch (own pass)
#   4. --pmc TCC_HIT_sum TCC_MISS_sum -> L2 hit rate per kernel (own pass)
# pmc_traffic.py stamps the summary with the kernel-source sha of this tree and
# $GIT_HEAD (pass the commit in the gpurun command: the box has no .git).
# MI355X_MICROARCH.md "HBM": FETCH_SIZE/WRITE_SIZE cannot share a pass, FETCH_SIZE
# is doubled on gfx950 (tools/pmc_traffic.py applies that).
# usage: tools/rocprof_bench.sh OUTDIR [bench.py args...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/$1
shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-count "$@" > "$OUT/bench_trace.json" 2> "$OUT/bench_trace.log" || exit $?
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-count "$@" > "$OUT/bench_fetch.json" 2> "$OUT/bench_fetch.log" || exit $?
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-count "$@" > "$OUT/bench_write.json" 2> "$OUT/bench_write.log" || exit $?
timeout -k 10 900 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/l2" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-count "$@" > "$OUT/bench_l2.json" 2> "$OUT/bench_l2.log" || exit $?
python3 "$R/tools/pmc_traffic.py" "$OUT" > "$OUT/pmc_traffic.json"
