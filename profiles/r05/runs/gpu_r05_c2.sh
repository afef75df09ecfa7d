set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c2
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_sim_pipeline.py tests/test_gpu_wide_cache.py tests/test_physics_analytic.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp CHROMA_BENCH_CACHE=/tmp/chroma_bench_cache
timeout -k 10 600 python3 $R/bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || exit $?
cut -c1-200 $O/bench.json
timeout -k 10 300 python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --sequential-steps 0 --timing-steps 0 --no-count > $O/bench_warm.json 2> $O/bench_warm.log || exit $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('warm setup', d['detail']['ranks'][0]['setup'], d['value'])" $O/bench_warm.json
