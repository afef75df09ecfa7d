#!/bin/bash
# Round-3 GPU pass (run through gpurun).  usage: tools/gpu_r03.sh TAG [tests|bench|prof|all] [pytest selection]
#   tests: smoke() + the -m gpu suite (or the given selection)
#   bench: the driver's bench command (20 timed / 5 warm-up)
#   prof:  rocprof kernel trace + PMC passes (tools/rocprof_bench.sh) -> stamped summary, then the bench
# Every GPU step has its own time limit; the first failure ends the script.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
TAG=$1
MODE=${2:-all}
SEL=${3:-tests}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R"
# progress marker for long single steps (a 29k-detector flatten + upload takes minutes
# with nothing else written); every GPU step below still has its own time limit
( while sleep 30; do date +%s > "$O/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
if [ "$MODE" = tests ] || [ "$MODE" = all ]; then
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
    tail -1 "$O/smoke.log"
    timeout -k 10 1500 python -u -m pytest $SEL -m gpu -x -v --timeout 1200 --timeout-method thread --durations=15 \
        > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
    tail -3 "$O/pytest_gpu.log"
fi
if [ "$MODE" = prof ]; then
    # kernel trace + FETCH/WRITE/L2 passes of the bench workload, stamped (GIT_HEAD from the caller)
    bash "$R/tools/rocprof_bench.sh" "gpurun_out/$TAG/prof" --steps 3 --warmup 1 || exit $?
    cp "$O/prof/pmc_traffic.json" "$R/profiles/latest_pmc.json" || exit $?
    # device region profile (libchroma_amd_prof.so)
    ( cd /tmp && export TMPDIR=/tmp && CHROMA_DEVICE_PROFILE=1 timeout -k 10 600 python3 "$R/bench.py" --steps 3 --warmup 1 \
        --no-cpu-baseline --no-count > "$O/devprof.json" 2> "$O/devprof.log" ) || { tail -5 "$O/devprof.log"; exit 1; }
fi
if [ "$MODE" = configs ]; then
    # the other BASELINE configs on one GPU (C3 primary geometry, C2, C5), 3 timed / 1 warm-up as in r02
    cd /tmp && export TMPDIR=/tmp
    for spec in "demo 10000000" "tiny 1000000" "scint 10000000"; do
        set -- $spec
        timeout -k 10 900 python3 "$R/bench.py" --detector $1 --photons $2 --steps 3 --warmup 1 \
            > "$O/bench_$1.json" 2> "$O/bench_$1.log" || { tail -20 "$O/bench_$1.log"; exit 1; }
        cut -c1-200 "$O/bench_$1.json"
    done
fi
if [ "$MODE" = bench ] || [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 900 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log" || { tail -20 "$O/bench.log"; exit 1; }
    cut -c1-400 "$O/bench.json"
fi
echo "gpu_r03 $TAG $MODE ok"
