# r06: photon-by-photon parity of the final kernels (sources 44368146) on more photon
# seeds: 29k seeds 7-22 (16 x 10 M photons), C5 scint and C3 demo seeds 1-4 (4 x 10 M
# each), every photon against the oracle (tools/parity_sweep.py)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_sweep2
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 -u "$R/tools/parity_sweep.py" 7,8,9,10,11,12,13,14,15,16,17,18,19,20,21,22 --photons 10000000 \
    > "$O/sweep_29k.jsonl" 2> "$O/sweep_29k.log" || { tail -20 "$O/sweep_29k.log"; exit 1; }
cut -c1-200 "$O/sweep_29k.jsonl" | tail -1
timeout -k 10 400 python3 -u "$R/tools/parity_sweep.py" 1,2,3,4 --detector scint --photons 10000000 \
    > "$O/sweep_scint.jsonl" 2> "$O/sweep_scint.log" || { tail -20 "$O/sweep_scint.log"; exit 1; }
cut -c1-200 "$O/sweep_scint.jsonl" | tail -1
timeout -k 10 400 python3 -u "$R/tools/parity_sweep.py" 1,2,3,4 --detector demo --photons 10000000 \
    > "$O/sweep_demo.jsonl" 2> "$O/sweep_demo.log" || { tail -20 "$O/sweep_demo.log"; exit 1; }
cut -c1-200 "$O/sweep_demo.jsonl" | tail -1
