set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_lone
mkdir -p $O
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 -u $R/tools/lone_walk_timing.py 29k > $O/lone_29k.jsonl 2> $O/lone_29k.log || { tail -20 $O/lone_29k.log; exit 1; }
cat $O/lone_29k.jsonl
