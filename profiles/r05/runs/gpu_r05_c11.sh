# tail grid on the tail stream (CHR_TAIL_GRID_DIV): batch tests, then the in-process A/B (29k, scintillator)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c11
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_batches.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_batches.log 2>&1 || { tail -30 $O/pytest_batches.log; exit 1; }
tail -1 $O/pytest_batches.log
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r05_ab_tailgrid "" - d1=CHR_TAIL_GRID_DIV:1 d2=CHR_TAIL_GRID_DIV:2 d4=CHR_TAIL_GRID_DIV:4 d8=CHR_TAIL_GRID_DIV:8 || exit 1
AB_ROUNDS=1 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab_tailgrid_c5 "" - d1=CHR_TAIL_GRID_DIV:1 d2=CHR_TAIL_GRID_DIV:2 d4=CHR_TAIL_GRID_DIV:4 || exit 1
