#!/bin/bash
# Device region profile on the GPU box: the profile-build parity/consistency test,
# then the bench workload under libchroma_amd_prof.so (CHROMA_DEVICE_PROFILE=1) and
# under the default library (same command), for the region table and its overhead.
# usage: tools/gpu_r02_devprof.sh TAG
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$1
mkdir -p "$O"
export CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_device_profile.py -m gpu -x -v --timeout 360 \
    --timeout-method thread > "$O/pytest_devprof.log" 2>&1
rc=$?
tail -3 "$O/pytest_devprof.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
CHROMA_DEVICE_PROFILE=1 timeout -k 10 400 python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-count \
    > "$O/bench_prof.json" 2> "$O/bench_prof.log" || { echo "prof bench failed"; tail -5 "$O/bench_prof.log"; exit 1; }
timeout -k 10 300 python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-count \
    > "$O/bench_default.json" 2> "$O/bench_default.log" || { echo "default bench failed"; tail -5 "$O/bench_default.log"; exit 1; }
python3 - "$O" <<'PY'
import json, sys
o = sys.argv[1]
for t in ('bench_prof', 'bench_default'):
    d = json.load(open('%s/%s.json' % (o, t)))
    print(t, round(d['value'] / 1e6, 1), 'M/s trace', round(d['detail']['trace_ms_per_step'], 2))
dp = json.load(open(o + '/bench_prof.json'))['detail']['device_profile']
khz = dp['clock_khz']
for k, v in dp['regions'].items():
    print('%-20s %14d calls %10.3f lane-s' % (k, v['calls'], v['cycles'] / (khz * 1e3) / 1e3))
PY
