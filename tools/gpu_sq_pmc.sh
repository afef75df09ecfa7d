#!/bin/bash
# SQ-counter pass of the bench workload (run through gpurun): issue vs wait
# cycles per dispatch of trace / shade / tail.  usage: tools/gpu_sq_pmc.sh TAG [env...]
# SQ_WANT="..." replaces the counter set (at most 8 SQ counters: one pass)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 120 rocprofv3 -L > "$O/counters.txt" 2>&1 || true
WANT=${SQ_WANT:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"}
[ $(echo $WANT | wc -w) -le 8 ] || { echo "more than 8 SQ counters"; exit 1; }
HAVE=""
for c in $WANT; do grep -qw "$c" "$O/counters.txt" && HAVE="$HAVE $c"; done
echo "counters:$HAVE"
[ -n "$HAVE" ] || exit 1
env "$@" timeout -s KILL 600 rocprofv3 --pmc $HAVE --output-format csv -d "$O/sq" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-count --steps 2 --warmup 1 > "$O/bench_sq.json" 2> "$O/bench_sq.log" \
    || { tail -20 "$O/bench_sq.log"; exit 1; }
echo "sq ok"
