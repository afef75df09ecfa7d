# r06: follow the BENCH_r05 mismatching photon (sample index 9043377 of 9,897,030)
# step by step on GPU and oracle (tools/parity_watch.py), then the SQ-counter pass
# of the bench workload (tools/gpu_sq_pmc.sh)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_watch
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
CHROMA_DEVICE_PROFILE=1 timeout -k 10 600 python3 -u "$R/tools/parity_watch.py" 9043377 --parity-photons 9897030 \
    > "$O/watch.json" 2> "$O/watch.log" || { tail -20 "$O/watch.log"; exit 1; }
cut -c1-1500 "$O/watch.json"
bash "$R/tools/gpu_sq_pmc.sh" r06_sq || exit 1
