set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c3
mkdir -p $O
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r05_ab1 "" - base= wo0=CHR_WALK_ORDER:0
