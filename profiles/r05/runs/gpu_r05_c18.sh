# first-step binning on / off (CHR_PROPAGATE_VARIANT 0 vs 8) at the current sources: 29k, scintillator
set -u
R=${GRAFT_REPO_ROOT}
cd $R
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r05_ab_bin "" - v0=CHR_PROPAGATE_VARIANT:0 v8=CHR_PROPAGATE_VARIANT:8 || exit 1
AB_ROUNDS=1 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab_bin_c5 "" - v0=CHR_PROPAGATE_VARIANT:0 v8=CHR_PROPAGATE_VARIANT:8 || exit 1
