# r06 round-end records, part 2: the driver's bench command (cold node-local cache,
# reading the PMC summary of part 1), then C2 / C3 / C5 bench lines
set -u
R=${GRAFT_REPO_ROOT}
TAG=${1:-r06_final}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 "$R/bench.py" --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log" || exit $?
cut -c1-300 "$O/bench.json"
cd "$R"
bash tools/bench_configs.sh gpurun_out/${TAG}_configs || exit 1
for f in gpurun_out/${TAG}_configs/*.json; do cut -c1-200 $f; done
