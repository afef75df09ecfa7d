set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/c5a; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reference_cases.py tests/test_gpu_configs.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 python3 $R/bench.py --detector scint --photons 10000000 --steps 3 --warmup 1 > $O/bench_scint.json 2> $O/bench_scint.log || { tail -20 $O/bench_scint.log; exit 1; }
cut -c1-200 $O/bench_scint.json
