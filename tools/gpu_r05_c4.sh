set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c4
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 python3 -u $R/bench.py --detector scint --photons 10000000 --steps 10 --warmup 3 > $O/bench_scint.json 2> $O/bench_scint.log || { tail -20 $O/bench_scint.log; exit 1; }
cut -c1-300 $O/bench_scint.json
