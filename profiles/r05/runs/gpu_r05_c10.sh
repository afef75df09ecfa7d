# early binning of the next batch (CHR_EARLY_BIN_SLOT) A/B, 29k then scintillator
set -u
R=${GRAFT_REPO_ROOT}
cd $R
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r05_ab_early "" - e0=CHR_EARLY_BIN_SLOT:0 e3=CHR_EARLY_BIN_SLOT:3 e5=CHR_EARLY_BIN_SLOT:5 e7=CHR_EARLY_BIN_SLOT:7 || exit 1
AB_ROUNDS=1 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab_early_c5 "" - e0=CHR_EARLY_BIN_SLOT:0 e5=CHR_EARLY_BIN_SLOT:5 || exit 1
