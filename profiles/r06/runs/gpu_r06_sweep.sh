# r06: photon-by-photon parity of the bench workload on six more photon seeds
# (tools/parity_sweep.py: 6 x 10 M photons, two pipelined batches each, vs the oracle)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_sweep
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 900 python3 -u "$R/tools/parity_sweep.py" 1,2,3,4,5,6 --photons 10000000 > "$O/sweep.jsonl" 2> "$O/sweep.log" \
    || { tail -20 "$O/sweep.log"; exit 1; }
cat "$O/sweep.jsonl" | cut -c1-300
