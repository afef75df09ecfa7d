# r06: the driver's bench command and the C5 line with bench.py's per-batch count of
# photons stopped at max_steps (detail.tail_launch[i].photons_at_max_steps; kernels
# unchanged, sources 44368146)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_maxsteps
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 "$R/bench.py" --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.log" || exit $?
cut -c1-200 "$O/bench.json"
timeout -k 10 600 python3 -u "$R/bench.py" --detector scint --photons 10000000 --steps 20 --warmup 5 \
    > "$O/bench_scint_10M.json" 2> "$O/bench_scint_10M.log" || exit $?
cut -c1-200 "$O/bench_scint_10M.json"
