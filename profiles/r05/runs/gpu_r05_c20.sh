# issue priority of draining trace waves (CHR_DRAIN_PRIO): A/B 29k, scintillator
set -u
R=${GRAFT_REPO_ROOT}
cd $R
AB_ROUNDS=2 bash tools/gpu_ab_env.sh r05_ab_dprio "" - d0=CHR_DRAIN_PRIO:0 d1=CHR_DRAIN_PRIO:1 d2=CHR_DRAIN_PRIO:2 d3=CHR_DRAIN_PRIO:3 || exit 1
AB_ROUNDS=1 AB_ARGS="--detector scint" bash tools/gpu_ab_env.sh r05_ab_dprio_c5 "" - d0=CHR_DRAIN_PRIO:0 d2=CHR_DRAIN_PRIO:2 || exit 1
