#!/bin/bash
# GPU A/B of env switches on the SEQUENTIAL path (one propagate call per step,
# the reference caller's loop): tools/ab_env.py with --no-pipeline.
# usage: tools/gpu_ab_seq.sh TAG STEPS CONFIG...
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; STEPS=$2; shift 2
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
( while sleep 30; do date +%s > "$O/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 1000 python3 -u "$R/tools/ab_env.py" --no-pipeline --steps "$STEPS" --warmup 2 -- "$@" > "$O/ab.jsonl" 2> "$O/ab.log" \
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
