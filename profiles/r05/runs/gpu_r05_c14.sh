# pair walk vs walk_lone in isolation (chr_walk_lone_timing)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_pair
mkdir -p $O
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 -u $R/tools/lone_walk_timing.py 29k > $O/pair_29k.jsonl 2> $O/pair_29k.log || { tail -20 $O/pair_29k.log; exit 1; }
cat $O/pair_29k.jsonl
