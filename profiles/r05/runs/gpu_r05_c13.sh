# long-lived photon's tail step split by phase (profile build): 29k and scintillator
set -u
R=${GRAFT_REPO_ROOT}
cd $R
bash tools/gpu_devprof.sh r05_long29k --steps 8 || exit 1
bash tools/gpu_devprof.sh r05_longc5 --detector scint --steps 6 || exit 1
