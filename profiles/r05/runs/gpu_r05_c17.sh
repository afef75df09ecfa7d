# pair walk, walker publishing after its node loads: timing in isolation, batch tests, A/B
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c17
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_batches.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
(cd /tmp && CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache timeout -k 10 600 python3 -u $R/tools/lone_walk_timing.py 29k > $O/pair_29k.jsonl 2> $O/pair_29k.log) || { tail -20 $O/pair_29k.log; exit 1; }
grep -v detector $O/pair_29k.jsonl
AB_ROUNDS=3 bash tools/gpu_ab_env.sh r05_ab_pair2 "" - p1=CHR_PAIR_WALK:1 p0=CHR_PAIR_WALK:0 || exit 1
