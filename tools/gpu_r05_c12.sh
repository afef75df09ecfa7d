# split first shade of a batch around the previous tail's RNG slots (CHR_SHADE_SPLIT): batch tests, then the in-process A/B (29k, scintillator)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c12
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_batches.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_batches.log 2>&1 || { tail -30 $O/pytest_batches.log; exit 1; }
tail -1 $O/pytest_batches.log
AB_ROUNDS=3 bash tools/gpu_ab_env.sh r05_ab_shadesplit "" - s1=CHR_SHADE_SPLIT:1 s0=CHR_SHADE_SPLIT:0 || exit 1
AB_ROUNDS=2 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab_shadesplit_c5 "" - s1=CHR_SHADE_SPLIT:1 s0=CHR_SHADE_SPLIT:0 || exit 1
