#!/bin/bash
# GPU A/B pass: a parity test subset, the driver's bench command (full line),
# then the same bench once per extra environment setting (bench only).
# usage (GPU box): tools/gpu_ab.sh TAG "pytest args" [ENV=VAL ...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; TESTS=$2; shift 2
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 600 --timeout-method thread > "$O/pytest.log" 2>&1
  rc=$?
  tail -6 "$O/pytest.log"
  [ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log"
rc=$?
echo "bench rc=$rc"; cut -c1-200 "$O/bench.json"
[ $rc -eq 0 ] || { tail -20 "$O/bench.log"; exit $rc; }
for kv in "$@"; do
  tag=$(echo "$kv" | tr '=' '_')
  env "$kv" timeout -k 10 400 python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-count \
      > "$O/bench_$tag.json" 2> "$O/bench_$tag.log"
  rc=$?
  echo "bench $kv rc=$rc"; cut -c1-200 "$O/bench_$tag.json"
  [ $rc -eq 0 ] || { tail -20 "$O/bench_$tag.log"; exit $rc; }
done
