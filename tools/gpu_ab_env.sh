#!/bin/bash
# GPU A/B of env switches (run through gpurun): optional parity tests under the
# first switch set, then tools/ab_env.py (one upload, interleaved rounds, photons
# hashed per configuration).
# usage: tools/gpu_ab_env.sh TAG "ENV=V ..." "pytest selection or -" CONFIG...
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; TENV=$2; TESTS=$3; shift 3
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
( while sleep 30; do date +%s > "$O/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
if [ "$TESTS" != "-" ]; then
  env $TENV timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 600 --timeout-method thread \
      > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 -u "$R/tools/ab_env.py" --steps 20 --warmup 5 ${AB_ARGS:-} -- "$@" > "$O/ab.jsonl" 2> "$O/ab.log" \
    || { tail -20 "$O/ab.log"; exit 1; }
python3 - "$O/ab.jsonl" <<'PY'
import json, sys, collections
acc = collections.defaultdict(list)
for line in open(sys.argv[1]):
    d = json.loads(line)
    if 'round' in d:
        acc[d['config']].append((d['photons_per_s'] / 1e6, d['trace_ms_per_step'], d['tail_ms_mean']))
    else:
        print(line.strip())
for k, v in acc.items():
    print(k, ' '.join('%.1fM/s trace %.2f tail %.2f' % x for x in v))
PY
