#!/bin/bash
# Device region profile of the bench workload (libchroma_amd_prof.so): one
# untimed propagate after a short bench run; the line's detail.device_profile.
# usage: tools/gpu_devprof.sh TAG [bench args]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=$1; shift
O=$R/gpurun_out/$T
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd /tmp && export TMPDIR=/tmp
CHROMA_DEVICE_PROFILE=1 timeout -k 10 600 python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-count \
    --sequential-steps 0 --timing-steps 0 "$@" > "$O/bench.json" 2> "$O/bench.log" || { tail -20 "$O/bench.log"; exit 1; }
python3 - "$O/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dp = d['detail']['device_profile']
json.dump(dp, open(sys.argv[1].replace('bench.json', 'device_profile.json'), 'w'), indent=1)
r = dp['regions']
khz = dp['clock_khz']
for k, v in r.items():
    if v['calls'] or v['cycles']:
        print('%-20s calls %12d cycles %16d' % (k, v['calls'], v['cycles']))
lw = r.get('lone_walk', {})
if lw.get('calls'):
    it = lw['calls']
    for k in ('lone_refill', 'lone_fetch', 'lone_expand', 'lone_tris'):
        print('%-12s %7.0f cycles/iteration (%.0f%%)' % (k, r[k]['cycles'] / it, 100.0 * r[k]['cycles'] / lw['cycles']))
    print('lone walk %.0f cycles/iteration = %.3f us at %d kHz' % (lw['cycles'] / it, lw['cycles'] / it / khz * 1e3, khz))
lg = r.get('long_walk', {})
if lg.get('calls'):
    n = lg['calls']
    tot = sum(r[k]['cycles'] for k in ('long_walk', 'long_fill', 'long_to_boundary', 'long_at_boundary', 'long_other'))
    for k in ('long_walk', 'long_fill', 'long_to_boundary', 'long_at_boundary', 'long_other'):
        print('%-17s %7.0f cycles/step = %6.3f us (%.0f%%)' % (k, r[k]['cycles'] / n, r[k]['cycles'] / n / khz * 1e3,
                                                          100.0 * r[k]['cycles'] / tot))
    print('long-lived photon step %.3f us over %d steps' % (tot / n / khz * 1e3, n))
PY
