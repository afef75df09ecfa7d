# r06: the lone climb's first iteration takes the start node's ancestors read during the
# previous step's physics: the GPU suite, then env A/B -- prefetch (default) vs none
# (CHR_WALK_UP=4), 29k and C5
set -u
R=${GRAFT_REPO_ROOT}
O=$R/gpurun_out/r06_f
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r06_ab_prefetch "" - pre= nopre=CHR_WALK_UP:4 || exit 1
AB_ROUNDS=1 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r06_ab_prefetch_c5 "" - pre= nopre=CHR_WALK_UP:4 || exit 1
