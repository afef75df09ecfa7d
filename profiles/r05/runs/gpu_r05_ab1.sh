# walk order A/B: 29k detector, then the scintillator detector (C5)
set -u
R=${GRAFT_REPO_ROOT}
cd $R
AB_ROUNDS=3 bash tools/gpu_ab_env.sh r05_ab1 "" - base= wo0=CHR_WALK_ORDER:0 || exit 1
AB_ROUNDS=2 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab1_c5 "" - base= wo0=CHR_WALK_ORDER:0 || exit 1
