# pair walk in the tail (CHR_PAIR_WALK): batch + parity tests, then the in-process A/B (29k, scintillator)
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c16
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_ROUNDS=3 bash tools/gpu_ab_env.sh r05_ab_pair "" - p1=CHR_PAIR_WALK:1 p0=CHR_PAIR_WALK:0 || exit 1
AB_ROUNDS=2 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab_pair_c5 "" - p1=CHR_PAIR_WALK:1 p0=CHR_PAIR_WALK:0 || exit 1
