# pipelined ray refills in trace_kernel (CHR_REFILL_PIPE): switch tests, A/B 29k + scintillator
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r05_c21
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_batches.py -m gpu -x -q --timeout 600 --timeout-method thread -k "switches or mirror or binned" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_ROUNDS=3 bash tools/gpu_ab_env.sh r05_ab_rpipe "" - r0=CHR_REFILL_PIPE:0 r1=CHR_REFILL_PIPE:1 || exit 1
AB_ROUNDS=2 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab_rpipe_c5 "" - r0=CHR_REFILL_PIPE:0 r1=CHR_REFILL_PIPE:1 || exit 1
