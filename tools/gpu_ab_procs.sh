#!/bin/bash
# GPU A/B of settings read when the geometry is built or the library loads
# (e.g. CHR_WIDE_LEAF_MAX, CHROMA_AMD_LIB): tools/ab_env.py once per setting and
# round, alternating, each in its own process.
# usage: tools/gpu_ab_procs.sh TAG ROUNDS "bench args" NAME=ENV:V,ENV:V NAME2= ...
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; ROUNDS=$2; BARGS=$3; shift 3
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
( while sleep 30; do date +%s > "$O/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
cd /tmp && export TMPDIR=/tmp
for r in $(seq 1 "$ROUNDS"); do
  for cfg in "$@"; do
    name=${cfg%%=*}; rest=${cfg#*=}
    envs=()
    IFS=',' read -ra kvs <<< "$rest"
    for kv in "${kvs[@]}"; do [ -n "$kv" ] && envs+=("${kv%%:*}=${kv#*:}"); done
    env "${envs[@]}" AB_ROUNDS=1 timeout -k 10 600 python3 -u "$R/tools/ab_env.py" $BARGS -- "$name=" \
        >> "$O/ab.jsonl" 2>> "$O/ab.log" || { tail -20 "$O/ab.log"; exit 1; }
  done
done
python3 - "$O/ab.jsonl" <<'PY'
import json, sys, collections, statistics as st
acc = collections.defaultdict(list)
for line in open(sys.argv[1]):
    d = json.loads(line)
    if 'round' in d:
        acc[d['config']].append('%.1fM/s trace %.2f tail %.2f long %.1f walk %.1f first %s' % (
            d['photons_per_s'] / 1e6, d['trace_ms_per_step'], d['tail_ms_mean'],
            st.median(d['long_us_per_step'] or [0]), st.median(d['long_walk_us_per_step'] or [0]),
            d['first_trace_launches_ms'][:3]))
    elif 'photons_sha' in d:
        print(d['config'], d['photons_sha'])
for k, v in acc.items():
    print(k, ' | '.join(v))
PY
