# r06: the device region profile of the final kernels (profile build, CHROMA_DEVICE_PROFILE=1):
# where the tail's long-lived photon's step goes after the climb (CHR_PROF_LONG_*), 29k and C5
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_dp
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache CHROMA_DEVICE_PROFILE=1
timeout -k 10 600 python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-count --sequential-steps 0 \
    > "$O/dp_29k.json" 2> "$O/dp_29k.log" || { tail -20 "$O/dp_29k.log"; exit 1; }
timeout -k 10 600 python3 "$R/bench.py" --detector scint --photons 10000000 --steps 3 --warmup 2 --no-cpu-baseline \
    --no-count --sequential-steps 0 > "$O/dp_scint.json" 2> "$O/dp_scint.log" || { tail -20 "$O/dp_scint.log"; exit 1; }
python3 - "$O/dp_29k.json" "$O/dp_scint.json" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    dp = d['detail'].get('device_profile', {})
    print(f.split('/')[-1], json.dumps({k: v for k, v in dp.get('regions', {}).items() if 'LONG' in k.upper() or 'TAIL' in k.upper()})[:1500])
PY
