# r06: the mismatching photon's second-step walk logged inside trace_kernel
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_watch2
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
WATCH_RAY=-1942.692138671875,16390.626953125,-1976.0341796875 CHROMA_DEVICE_PROFILE=1 timeout -k 10 600 \
    python3 -u "$R/tools/parity_watch.py" 9043377 --parity-photons 9897030 > "$O/watch.json" 2> "$O/watch.log" \
    || { tail -20 "$O/watch.log"; exit 1; }
cut -c1-600 "$O/watch.json"
